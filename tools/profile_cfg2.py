"""cfg2 (d=8 cfg2 distributions, native LHS fused into the inverse CDFs, no correlation) through
Node.sample_device: wall time per call at N=1e7 and at N=1e3 (host and launch overhead alone),
the device time of each timed kernel per call (pbh_timing) and a cProfile of the small calls.
python tools/profile_cfg2.py [calls]"""
import cProfile
import ctypes
import json
import pstats
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.pipeline import cfg_dists  # noqa: E402
from probabilit_amd import _lib, device  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = device.device()
lib = _lib.load()
ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
root = NoOp(*ds)
out = {}
for n in (10_000_000, 1_000):
    for i in range(3):
        root.sample_device(n, random_state=i, method="lhs")
    torch.cuda.synchronize(dev)
    lib.pbh_timing_reset()
    lib.pbh_timing_enable(1)
    t = time.perf_counter()
    for i in range(calls):
        root.sample_device(n, random_state=100 + i, method="lhs")
    torch.cuda.synchronize(dev)
    wall = (time.perf_counter() - t) / calls
    lib.pbh_timing_enable(0)
    ker = {}
    for kid, name in enumerate(_lib.KERNELS):
        tt, c = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(tt), ctypes.byref(c)))
        if c.value:
            ker[name] = {"ms_per_call": round(tt.value / calls, 4), "launches_per_call": c.value / calls}
    out[str(n)] = {"wall_ms_per_call": round(1e3 * wall, 3), "kernels": ker}
    # untimed wall (timing events off)
    t = time.perf_counter()
    for i in range(calls):
        root.sample_device(n, random_state=200 + i, method="lhs")
    torch.cuda.synchronize(dev)
    out[str(n)]["wall_ms_untimed"] = round(1e3 * (time.perf_counter() - t) / calls, 3)
print(json.dumps(out, indent=1), flush=True)
pr = cProfile.Profile()
pr.enable()
for i in range(calls):
    root.sample_device(1_000, random_state=300 + i, method="lhs")
pr.disable()
torch.cuda.synchronize(dev)
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
st.sort_stats("cumulative").print_stats(40)
