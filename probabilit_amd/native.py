"""Thin numpy/torch front-ends for single native kernels (used by tests, bench and callers
that want one kernel without building a DAG).  Each wraps one C-ABI entry point."""

import numpy as np

from . import _lib, device
from .modeling import _DIST_SHAPES, _parse_scipy_args


def _dev_vec(a):
    import torch

    if isinstance(a, torch.Tensor):
        return a.to(device.device(), torch.float64).contiguous()
    return device.to_device(np.ascontiguousarray(a, dtype=np.float64))


def _params(name, n, kwargs):
    out, keep = [], []
    for v in _parse_scipy_args(name, (), kwargs):
        a = np.asarray(v) if not hasattr(v, "data_ptr") else None
        if a is not None and a.ndim == 0:
            out.append(_lib.Param(None, float(a)))
        else:
            t = _dev_vec(v)
            assert t.shape == (n,)
            keep.append(t)
            out.append(_lib.Param(t.data_ptr(), 0.0))
    return (_lib.Param * len(out))(*out), keep


def ppf(name, q, return_device=False, **params):
    """scipy.stats.<name>(**params).ppf(q) on the GPU (pbh_ppf)."""
    if name not in _DIST_SHAPES:
        raise NotImplementedError(name)
    qd = _dev_vec(q)
    n = qd.shape[0]
    arr, keep = _params(name, n, params)
    out = device.empty(n)
    flag = device.zeros(1, "int32")
    _lib.check(_lib.load().pbh_ppf(_lib.DIST_IDS[name], qd.data_ptr(), 1, n, arr, len(arr), out.data_ptr(),
                                   flag.data_ptr(), device.stream()), "pbh_ppf")
    del keep
    return out if return_device else device.to_host(out)


def lhs_ppf(name, seed, n_total, col, row0=0, nrows=None, return_device=False, **params):
    """Fused native-LHS column `col` of an n_total-row design pushed through ppf (pbh_lhs_ppf).
    (n_total, not n: binom's shape parameter is called n.)"""
    nrows = n_total - row0 if nrows is None else nrows
    arr, keep = _params(name, nrows, params)
    out = device.empty(nrows)
    _lib.check(_lib.load().pbh_lhs_ppf(seed, n_total, row0, nrows, col, _lib.DIST_IDS[name], arr, len(arr),
                                       out.data_ptr(), None, device.stream()), "pbh_lhs_ppf")
    del keep
    return out if return_device else device.to_host(out)


def fill_lhs(seed, n, d, row0=0, nrows=None, return_device=False):
    """(nrows, d) native Latin hypercube rows [row0, row0 + nrows) (column-major on device)."""
    nrows = n - row0 if nrows is None else nrows
    q = device.empty((d, nrows))
    _lib.check(_lib.load().pbh_fill_lhs(seed, n, row0, nrows, 0, d, q.data_ptr(), nrows, device.stream()),
               "pbh_fill_lhs")
    return q if return_device else device.to_host(q).T


def fill_uniform(seed, n, d, row0=0, return_device=False):
    q = device.empty((d, n))
    _lib.check(_lib.load().pbh_fill_uniform(seed, row0, n, 0, d, q.data_ptr(), n, device.stream()),
               "pbh_fill_uniform")
    return q if return_device else device.to_host(q).T


def fill_sobol(sv, shift, n, bits=30, row0=0, return_device=False):
    sv = np.ascontiguousarray(sv, dtype=np.uint32)
    shift = np.ascontiguousarray(shift, dtype=np.uint32)
    d = sv.shape[0]
    q = device.empty((d, n))
    _lib.check(_lib.load().pbh_fill_sobol(_lib.np_ptr(sv), _lib.np_ptr(shift), d, bits, row0, n, 0, d, q.data_ptr(),
                                          n, device.stream()), "pbh_fill_sobol")
    return q if return_device else device.to_host(q).T


def transpose(x_dev, rows, cols):
    out = device.empty((cols, rows))
    _lib.check(_lib.load().pbh_transpose(x_dev.data_ptr(), rows, cols, cols, out.data_ptr(), rows,
                                         device.stream()), "pbh_transpose")
    return out

