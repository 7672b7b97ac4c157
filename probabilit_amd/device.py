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
    return t.detach().cpu().numpy()


def ptr(t):
    return None if t is None else t.data_ptr()


def synchronize():
    _torch().cuda.synchronize(device())


_TORCH = {"float64": "float64", "int64": "int64", "bool": "bool", "int32": "int32", "uint8": "uint8",
          "uint32": "int32"}
