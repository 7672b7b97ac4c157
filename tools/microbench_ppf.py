"""Per-distribution device time of the fused native-LHS inverse-CDF kernel (pbh_lhs_ppf) and
of the stratum-ordered variant, N rows per launch (HIP events on the launching stream).

    python tools/microbench_ppf.py [--n 100000000] [--reps 3]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    from probabilit_amd import device, native

    device.device()
    cases = [("norm", {"loc": 0.0, "scale": 1.0}), ("gamma", {"a": 2.0}), ("gamma", {"a": 0.7, "scale": 3.0}),
             ("triang", {"c": 0.3}), ("poisson", {"mu": 4.0}), ("poisson", {"mu": 30.0}), ("expon", {}),
             ("uniform", {}), ("lognorm", {"s": 0.5})]
    out = {}
    for name, kw in cases:
        native.lhs_ppf(name, 1, a.n, 0, return_device=True, **kw)  # warm
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for r in range(a.reps):
            native.lhs_ppf(name, 1 + r, a.n, r, return_device=True, **kw)
        ev1.record()
        torch.cuda.synchronize()
        ms = ev0.elapsed_time(ev1) / a.reps
        out[f"{name}{kw}"] = {"ms": round(ms, 3), "GBps_write": round(8 * a.n / ms / 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
