"""D2H hand-back options for `.samples_` (device columns -> fresh numpy arrays), measured on the
box: pageable copy, a pinned allocation per call, pinned staging chunks + threaded memcpy into a
fresh pageable array, and hipHostRegister of the destination.  python tools/d2h_bench.py [GB]"""

import ctypes
import json
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def main():
    gb = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    n = int(gb * (1 << 30)) // 8
    dev = torch.device("cuda", 0)
    src = torch.empty(n, dtype=torch.float64, device=dev).normal_()
    torch.cuda.synchronize()
    out = {"bytes": n * 8}

    def rate(t):
        return round(n * 8 / t / 1e9, 2)

    # (a) pageable: what device.to_host does today
    t0 = time.perf_counter()
    a = src.cpu().numpy()
    out["pageable_GBps"] = rate(time.perf_counter() - t0)
    del a

    # (b) pinned allocation per call + one DMA
    t0 = time.perf_counter()
    h = torch.empty(n, dtype=torch.float64, pin_memory=True)
    t1 = time.perf_counter()
    h.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    out["pinned_alloc_s"] = round(t1 - t0, 3)
    out["pinned_dma_GBps"] = rate(t2 - t1)
    out["pinned_total_GBps"] = rate(t2 - t0)
    del h

    # (c) staging ring of pinned chunks + threaded memcpy into a fresh pageable array
    import mmap

    try:
        out["thp"] = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
    except OSError:
        out["thp"] = None

    def huge_empty(m):  # an anonymous mapping advised for transparent huge pages
        mm = mmap.mmap(-1, m * 8, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        try:
            mm.madvise(mmap.MADV_HUGEPAGE)
        except (AttributeError, OSError):
            pass
        return np.frombuffer(mm, dtype=np.float64, count=m)

    for chunk_mb, threads, alloc in ((64, 16, "np"), (64, 16, "huge"), (64, 16, "prefault"), (32, 16, "huge"),
                                     (128, 16, "huge")):
        chunk = chunk_mb * (1 << 20) // 8
        ring = [torch.empty(chunk, dtype=torch.float64, pin_memory=True) for _ in range(3)]
        evs = [torch.cuda.Event() for _ in range(3)]
        stream = torch.cuda.Stream(device=dev)
        pool = ThreadPoolExecutor(threads)
        if alloc == "prefault":
            dst = np.empty(n, dtype=np.float64)
            dst[:] = 0.0
        t0 = time.perf_counter()
        if alloc == "np":
            dst = np.empty(n, dtype=np.float64)
        elif alloc == "huge":
            dst = huge_empty(n)
        nch = (n + chunk - 1) // chunk

        def copy_out(i, slot):
            lo = i * chunk
            hi = min(n, lo + chunk)
            v = ring[slot].numpy()[:hi - lo]
            # split the chunk over the threads: parallel memcpy into the (first-touched) destination
            parts = threads
            step = (hi - lo + parts - 1) // parts
            list(pool.map(lambda j: np.copyto(dst[lo + j * step:min(hi, lo + (j + 1) * step)],
                                              v[j * step:min(hi - lo, (j + 1) * step)]), range(parts)))

        with torch.cuda.stream(stream):
            for i in range(nch + 2):
                if i < nch:  # DMA of chunk i into its slot (free: chunk i - 3 was copied out)
                    slot = i % 3
                    lo = i * chunk
                    hi = min(n, lo + chunk)
                    ring[slot][:hi - lo].copy_(src[lo:hi], non_blocking=True)
                    evs[slot].record(stream)
                j = i - 2  # chunk j's DMA was issued two chunks ago: wait for it, copy it out
                if 0 <= j < nch:
                    evs[j % 3].synchronize()
                    copy_out(j, j % 3)
        t = time.perf_counter() - t0
        assert np.array_equal(dst[:1000], src[:1000].cpu().numpy())
        out[f"ring_{chunk_mb}MB_{threads}t_{alloc}_GBps"] = rate(t)
        pool.shutdown()
        del dst, ring

    # (d) hipHostRegister of a fresh pageable destination, then one DMA
    hip = ctypes.CDLL("libamdhip64.so")
    t0 = time.perf_counter()
    dst = np.empty(n, dtype=np.float64)
    st = hip.hipHostRegister(ctypes.c_void_p(dst.ctypes.data), ctypes.c_size_t(n * 8), 0)
    t1 = time.perf_counter()
    if st == 0:
        hv = torch.from_numpy(dst)
        hv.copy_(src, non_blocking=False)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        hip.hipHostUnregister(ctypes.c_void_p(dst.ctypes.data))
        t3 = time.perf_counter()
        out["register_s"] = round(t1 - t0, 3)
        out["register_dma_GBps"] = rate(t2 - t1)
        out["register_total_GBps"] = rate(t3 - t0)
    else:
        out["register_error"] = st
    print(json.dumps(out))


if __name__ == "__main__":
    main()
