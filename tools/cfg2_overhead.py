"""Where cfg2's per-call time goes at small N (host overhead): the whole Node.sample_device,
the one grouped C call alone (pbh_lhs_ppf_columns, no graph work), and the graph work alone.
python tools/cfg2_overhead.py [n] [calls]"""
import ctypes
import json
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from oracle.pipeline import cfg_dists  # noqa: E402
from probabilit_amd import _lib, device  # noqa: E402
from probabilit_amd.modeling import Distribution, NoOp, _parse_scipy_args  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
dev = device.device()
lib = _lib.load()
ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
root = NoOp(*ds)
out = {"n": n}


def timeit(fn):
    for _ in range(5):
        fn()
    torch.cuda.synchronize(dev)
    t = time.perf_counter()
    for _ in range(calls):
        fn()
    torch.cuda.synchronize(dev)
    return round(1e6 * (time.perf_counter() - t) / calls, 1)


out["sample_device_us"] = timeit(lambda: root.sample_device(n, random_state=1, method="lhs"))
flags = torch.zeros(16, dtype=torch.int32, device=dev)
cols = []
for j, d in enumerate(ds):
    params = [float(v) for v in _parse_scipy_args(d.distr, d.args, d.kwargs)]
    cols.append(_lib.ICColumn(7, j, _lib.DIST_IDS[d.distr], (ctypes.c_double * 4)(*(params + [0.0] * (4 - len(params)))),
                              len(params), flags.data_ptr() + 4 * j))
arr = (_lib.ICColumn * len(cols))(*cols)
blk = device.empty((len(cols), n))


def grouped():
    _lib.check(lib.pbh_lhs_ppf_columns(arr, len(cols), n, 0, n, blk.data_ptr(), n, device.stream()))


out["grouped_call_us"] = timeit(grouped)


def grouped_sync():
    grouped()
    flags.cpu()


out["grouped_call_plus_readback_us"] = timeit(grouped_sync)
t = time.perf_counter()
for _ in range(calls):
    grouped()
out["grouped_call_host_only_us"] = round(1e6 * (time.perf_counter() - t) / calls, 1)
torch.cuda.synchronize(dev)
t = time.perf_counter()
for _ in range(calls):
    G = root.to_graph()
out["to_graph_us"] = round(1e6 * (time.perf_counter() - t) / calls, 1)
print(json.dumps(out), flush=True)
