"""Step 3 alone (pbh_ic_apply, no step-4 codes) on N=1e8 x K=32 device scores, HIP-event time of
k_apply: compares with the bench's k_apply, which also writes the 32-bit codes.

    python tools/microbench_apply.py
"""

import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from oracle.pipeline import cfg3_corr
    from probabilit_amd import _lib, device
    from probabilit_amd.distributed import HipPhases

    device.device()
    n, k = 100_000_000, 32
    S = torch.randn((k, n), dtype=torch.float64, device="cuda")
    C = cfg3_corr(k)
    P = np.linalg.cholesky(C)
    L = np.linalg.cholesky(np.corrcoef(np.random.default_rng(0).normal(size=(1000, k)), rowvar=False))
    ph = HipPhases()
    lib = _lib.load()
    ph.apply(S, L, P)
    lib.pbh_timing_reset()
    lib.pbh_timing_enable(1)
    for _ in range(3):
        ph.apply(S, L, P)
    lib.pbh_timing_enable(0)
    t, c = ctypes.c_double(), ctypes.c_int64()
    _lib.check(lib.pbh_timing_read(_lib.KERNELS.index("k_apply"), ctypes.byref(t), ctypes.byref(c)))
    ms = t.value / c.value
    print(json.dumps({"k_apply_no_codes_ms": round(ms, 3), "GBps": round(16 * n * k / ms / 1e6, 1)}))


if __name__ == "__main__":
    main()
