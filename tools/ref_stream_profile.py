"""The same-seed side figure's workload (cfg3 graph at N=1e7 on stream="reference") for a
kernel-trace profile: python tools/ref_stream_profile.py [calls]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.pipeline import cfg3_corr, cfg_dists  # noqa: E402
from probabilit_amd import device  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2
dev = device.device()
ds = [Distribution(name, **kw) for name, kw in cfg_dists(32)]
root = NoOp(*ds).correlate(*ds, corr_mat=cfg3_corr(32))
root.sample_device(10_000_000, random_state=1, method="lhs", stream="reference")
torch.cuda.synchronize(dev)
for i in range(calls):
    t = time.perf_counter()
    root.sample_device(10_000_000, random_state=2 + i, method="lhs", stream="reference")
    torch.cuda.synchronize(dev)
    print(f"call {i}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
