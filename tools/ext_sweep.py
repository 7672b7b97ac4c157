"""Inverse-CDF sweep times of the extended distributions (pbh_ppf over an HBM-resident quantile
column, HIP events via pbh_timing, best of 3 after a warm call) and the correlated-PERT fast
path end to end: python tools/ext_sweep.py [rows [variant]] (variant: a library built by
build.py --variant)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import probabilit_amd  # noqa: E402,F401
from probabilit_amd import _lib, device, native  # noqa: E402

if len(sys.argv) > 2:
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), f"libprobabilit_hip_{sys.argv[2]}.so")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    lib = _lib.load()
    q = native.fill_uniform(7, n, 1, return_device=True)[0]
    kid = _lib.KERNELS.index("k_ppf")
    out = {"rows": n, "sweep_ms": {}}
    cases = [("norm", {}), ("beta", dict(a=3.4, b=2.6, scale=10.0)), ("beta", dict(a=0.5, b=0.5)),
             ("truncnorm", dict(a=-1.0, b=2.0)), ("binom", dict(n=20, p=0.3)), ("weibull_min", dict(c=1.7)),
             ("chi", dict(df=3.0)), ("burr12", dict(c=2.0, d=3.0)), ("trapezoid", dict(c=0.2, d=0.8)),
             ("bernoulli", dict(p=0.3)), ("maxwell", {}), ("nakagami", dict(nu=4.97)), ("chi2", dict(df=5.5)),
             ("nbinom", dict(n=3.5, p=0.4)), ("geom", dict(p=0.3)), ("randint", dict(low=2, high=40)),
             ("invgamma", dict(a=2.5)), ("t", dict(df=4.0))]
    for name, kw in cases:
        native.ppf(name, q, return_device=True, **kw)
        ms = []
        for _ in range(3):
            import ctypes

            lib.pbh_timing_reset()
            lib.pbh_timing_enable(1)
            native.ppf(name, q, return_device=True, **kw)
            lib.pbh_timing_enable(0)
            t, c = ctypes.c_double(), ctypes.c_int64()
            _lib.check(lib.pbh_timing_read(kid, ctypes.byref(t), ctypes.byref(c)))
            ms.append(t.value / max(c.value, 1))
        out["sweep_ms"][f"{name}{kw}"] = round(min(ms), 4)
    # correlated PERT through the generated-column path, device-resident output
    from probabilit_amd import distributions as dists
    from probabilit_amd.modeling import NoOp

    d = 8
    ds = [dists.PERT(0, 1 + j, 10 + j) for j in range(d)]
    C = 0.5 * np.eye(d) + 0.5
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    root.sample_device(n, random_state=0, method="lhs")
    device.synchronize()
    t0 = time.perf_counter()
    root.sample_device(n, random_state=1, method="lhs")
    device.synchronize()
    out["pert_ic_ms"] = {"rows": n, "d": d, "ms": round((time.perf_counter() - t0) * 1e3, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
