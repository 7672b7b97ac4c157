"""The bench's side workloads, one stream (pbh_set_serial), for a rocprofv3 kernel-trace summary:

    python tools/side_profile.py operator  [rows] [calls]   # ImanConover().set_target(C)(X), X (rows, 32)
    python tools/side_profile.py refstream [rows] [calls]   # cfg3 graph on stream="reference"

bench.py's `operator_ic.rocprof` / `reference_stream.at_rows.dominant_kernel` read the committed
summaries (profiles/r*/rocprof_<workload>_*.csv)."""
import sys
import time

import numpy as np  # noqa: F401
import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import probabilit_amd  # noqa: E402,F401
from oracle.pipeline import cfg3_corr, cfg_dists  # noqa: E402
from probabilit_amd import _lib, device  # noqa: E402
from probabilit_amd.correlation import ImanConover  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp  # noqa: E402

what = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100_000_000
calls = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = device.device()
lib = _lib.load()
ds = [Distribution(name, **kw) for name, kw in cfg_dists(32)]
C = cfg3_corr(32)
lib.pbh_set_serial(1)
if what == "operator":
    NoOp(*ds).sample_device(n, random_state=3, method="lhs")
    X = torch.stack([x.samples_device for x in ds], dim=1)
    for x in ds:
        del x.samples_
    inst = ImanConover().set_target(C)
    run = lambda i: inst(X)  # noqa: E731
else:
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    run = lambda i: root.sample_device(n, random_state=5 + i, method="lhs", stream="reference")  # noqa: E731
for i in range(calls):
    t = time.perf_counter()
    out = run(i)
    torch.cuda.synchronize(dev)
    del out
    print(f"{what} call {i}: {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
