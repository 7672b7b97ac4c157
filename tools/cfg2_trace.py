"""cfg2 (d=8, native LHS fused into the inverse CDFs, no correlation) at N=1e7, repeated for a
kernel trace: python tools/cfg2_trace.py [calls]"""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.pipeline import cfg_dists  # noqa: E402
from probabilit_amd import device  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = device.device()
ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
root = NoOp(*ds)
for i in range(3):
    root.sample_device(10_000_000, random_state=i, method="lhs")
torch.cuda.synchronize(dev)
t = time.perf_counter()
for i in range(calls):
    root.sample_device(10_000_000, random_state=100 + i, method="lhs")
torch.cuda.synchronize(dev)
print(f"wall {1e3 * (time.perf_counter() - t) / calls:.3f} ms per call", flush=True)
