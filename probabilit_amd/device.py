"""Device plumbing: PyTorch-ROCm provides HBM allocations and the HIP stream; all compute
goes through libprobabilit_hip (probabilit_amd._lib).

One process drives one GPU.  The device is `cuda:<LOCAL_RANK>` under torch.distributed
launchers, else the current torch device.  There is no CPU fallback: without a visible
gfx950 GPU every sampling entry point raises RuntimeError.
"""

import os

import numpy as np

from . import _lib

_state = {"device": None}


def _torch():
    import torch

    return torch


def device():
    """The torch.device all samples live on (initialises the native library once)."""
    if _state["device"] is not None:
        return _state["device"]
    torch = _torch()
    if not torch.cuda.is_available():
        raise RuntimeError("probabilit_amd needs an AMD Instinct MI355X (gfx950) GPU; none is visible "
                           "(torch.cuda.is_available() is False). There is no CPU fallback.")
    idx = int(os.environ.get("LOCAL_RANK", torch.cuda.current_device()))
    idx = idx % torch.cuda.device_count()
    torch.cuda.set_device(idx)
    lib = _lib.load()
    _lib.check(lib.pbh_init(idx), "pbh_init")
    _state["device"] = torch.device("cuda", idx)
    return _state["device"]


def stream():
    """Raw hipStream_t of torch's current stream (what every pbh_* call is ordered on)."""
    return _torch().cuda.current_stream(device()).cuda_stream


def empty(n, dtype="float64"):
    torch = _torch()
    return torch.empty(n, dtype=getattr(torch, _TORCH[np.dtype(dtype).name]), device=device())


def zeros(n, dtype="float64"):
    torch = _torch()
    return torch.zeros(n, dtype=getattr(torch, _TORCH[np.dtype(dtype).name]), device=device())


def to_device(a):
    """Upload a numpy array (or pass through a device tensor)."""
    torch = _torch()
    if isinstance(a, torch.Tensor):
        return a.to(device())
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a).to(device(), non_blocking=False)


def to_host(t):
    """Download a device tensor to a fresh numpy array (synchronises the stream)."""
    return to_host_many([t])[0]


# The hand-back of samples_ to numpy (modeling.py:582-583, 614: the reference returns host
# arrays).  A pageable D2H runs at ~8-11 GB/s on the box (the runtime stages it through its own
# small pinned buffers, one chunk at a time); pinning a fresh destination per call costs ~0.07 s
# per GB.  Instead: a ring of three 128 MiB pinned buffers kept for the process, DMA of chunk i
# into one while the host threads copy chunk i - 2 out into the fresh numpy array (first touch
# included): 54.7 GB/s on 8 GiB, against 48.5 with 64 MiB chunks, 42 with 32 MiB, and 49.9 with
# the destination pre-faulted (so page faults are not the limit) (tools/d2h_bench.py,
# profiles/r03/d2h_r3b.json).
_STAGE_BYTES = 128 << 20
_SMALL_BYTES = 8 << 20  # below this a plain copy is as fast
_stage = {}
_stage_lock = __import__("threading").Lock()  # one user of the ring at a time (callers may be threads)


def _staging():
    if not _stage:
        import concurrent.futures

        torch = _torch()
        dev = device()
        _stage["ring"] = [torch.empty(_STAGE_BYTES, dtype=torch.uint8, pin_memory=True) for _ in range(3)]
        _stage["events"] = [torch.cuda.Event() for _ in range(3)]
        _stage["stream"] = torch.cuda.Stream(device=dev)
        _stage["threads"] = max(1, min(16, os.cpu_count() or 1))
        _stage["pool"] = concurrent.futures.ThreadPoolExecutor(_stage["threads"])
    return _stage


def to_host_many(tensors):
    """Fresh numpy copies of device tensors, the large ones pipelined through the pinned ring."""
    torch = _torch()
    outs = [None] * len(tensors)
    chunks = []  # (source bytes, destination bytes, lo, hi)
    for j, t in enumerate(tensors):
        t = t.detach()
        nbytes = t.numel() * t.element_size()
        if nbytes < _SMALL_BYTES or t.dtype == torch.bool or not t.is_contiguous():
            outs[j] = t.cpu().numpy()
            continue
        out = np.empty(tuple(t.shape), dtype=np.dtype(str(t.dtype).replace("torch.", "")))
        outs[j] = out
        src = t.reshape(-1).view(torch.uint8)
        dst = out.reshape(-1).view(np.uint8)
        for lo in range(0, nbytes, _STAGE_BYTES):
            chunks.append((src, dst, lo, min(nbytes, lo + _STAGE_BYTES)))
    if not chunks:
        return outs
    with _stage_lock:
        _drain_chunks(chunks)
    return outs


def _drain_chunks(chunks):
    torch = _torch()
    st = _staging()
    ring, evs, stream, pool, nt = st["ring"], st["events"], st["stream"], st["pool"], st["threads"]
    stream.wait_stream(torch.cuda.current_stream(device()))  # after the producers of the tensors

    def drain(i):
        src, dst, lo, hi = chunks[i]
        evs[i % 3].synchronize()
        buf = ring[i % 3].numpy()
        step = -(-(hi - lo) // nt)
        step = (step + 63) // 64 * 64
        list(pool.map(lambda a: np.copyto(dst[lo + a:min(hi, lo + a + step)], buf[a:min(hi - lo, a + step)]),
                      range(0, hi - lo, step)))

    with torch.cuda.stream(stream):
        for i in range(len(chunks) + 2):
            if i < len(chunks):  # slot i % 3 is free: chunk i - 3 was drained two iterations ago
                src, dst, lo, hi = chunks[i]
                ring[i % 3][:hi - lo].copy_(src[lo:hi], non_blocking=True)
                evs[i % 3].record(stream)
            if i >= 2:
                drain(i - 2)
    # every chunk was drained: no DMA still reads a source


def ptr(t):
    return None if t is None else t.data_ptr()


def synchronize():
    _torch().cuda.synchronize(device())


def clear_table_cache():
    """Free the process cache of inverse-CDF setup tables (gamma / beta guides, poisson / binom /
    nbinom CDF tables kept between calls, pbh_table_cache.hip): every table no call holds, after
    the kernels that read it.  Returns (freed, kept).  The cache is bounded anyway (1 GiB, LRU,
    tables over 64 MiB never kept); this returns its HBM to the caller between workloads."""
    import ctypes

    from . import _lib

    device()
    freed, kept = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.load().pbh_table_cache_clear(ctypes.byref(freed), ctypes.byref(kept)), "pbh_table_cache_clear")
    return freed.value, kept.value


_TORCH = {"float64": "float64", "int64": "int64", "bool": "bool", "int32": "int32", "uint8": "uint8",
          "uint32": "int32"}
