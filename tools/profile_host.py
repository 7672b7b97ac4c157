"""Host-side profile of the cfg3 bench step (bench.py's `step`): wall time per call against the
device time between its first and last kernel is not visible here, so this prints the Python
cProfile of a few warm calls (cumulative) and the wall time of each call.
python tools/profile_host.py [rows] [calls]"""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from probabilit_amd import device  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 3
d = 32
base = [("norm", {"loc": 0.0, "scale": 1.0}), ("gamma", {"a": 2.0}), ("triang", {"c": 0.3}), ("poisson", {"mu": 4.0}),
        ("norm", {"loc": 5.0, "scale": 2.0}), ("gamma", {"a": 0.7, "scale": 3.0}),
        ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}), ("poisson", {"mu": 30.0})]
dists = (base * 4)[:d]
A = np.random.default_rng(0).normal(size=(64, d))
C = 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(d)
ds = [Distribution(name, **kw) for name, kw in dists]
root = NoOp(*ds).correlate(*ds, corr_mat=C)
dev = device.device()
for i in range(2):
    root.sample_device(n, random_state=i, method="lhs")
torch.cuda.synchronize(dev)
pr = cProfile.Profile()
for i in range(calls):
    t = time.perf_counter()
    pr.enable()
    root.sample_device(n, random_state=10 + i, method="lhs")
    pr.disable()
    torch.cuda.synchronize(dev)
    print(f"call {i}: {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(45)
