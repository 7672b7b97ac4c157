"""Timing of the reference LHS stream (stream="reference") at n x d: the device decode's wall
time per call, its attempts and ambiguous-draw count, against the host shuffles.
python tools/ref_lhs_time.py [n] [d] [reps] [variant]"""
import ctypes
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from probabilit_amd import _lib, device, qmc  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
d = int(sys.argv[2]) if len(sys.argv) > 2 else 32
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
if len(sys.argv) > 4 and sys.argv[4] != "default":  # a library variant (build.py --variant) for A/B runs
    import os
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), f"libprobabilit_hip_{sys.argv[4]}.so")
dev = device.device()
lib = _lib.load()


def stats():
    a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    _lib.check(lib.pbh_lhs_reference_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
    return a.value, b.value, c.value


out = {"n": n, "d": d, "runs": []}
for r in range(reps):
    src = qmc.make_source("lhs", n, d, 1000 + r, stream="reference")
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    q = src.matrix()
    torch.cuda.synchronize(dev)
    ms = 1e3 * (time.perf_counter() - t)
    dv, att, amb = stats()
    out["runs"].append({"ms": round(ms, 2), "Msamples_per_s": round(n * d / ms / 1e3, 1), "device": dv,
                        "attempts": att, "ambiguous": amb})
    print(json.dumps(out["runs"][-1]), flush=True)
if n * d <= 40_000_000:  # check the last matrix against the host shuffles
    import scipy.stats
    ref = scipy.stats.qmc.LatinHypercube(d=d, rng=1000 + reps - 1).random(n)
    out["equal_to_scipy"] = bool(np.array_equal(device.to_host(q).T, ref))
print(json.dumps(out), flush=True)
