"""The bench's ppf-sweep side measurement on its own (pbh_ppf over an HBM-resident q column,
16 B per draw, HIP-event time of k_ppf on the launching stream), for A/B runs of the kernels:

    python tools/ppf_sweep.py [--rows 100000000]
"""

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--variant", default=None, help="load libprobabilit_hip_<variant>.so (build.py --variant)")
    a = ap.parse_args()
    import bench
    from probabilit_amd import _lib, device

    if a.variant:
        _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), f"libprobabilit_hip_{a.variant}.so")

    device.device()
    base = [("norm", {"loc": 0.0, "scale": 1.0}), ("gamma", {"a": 2.0}), ("triang", {"c": 0.3}),
            ("poisson", {"mu": 4.0}), ("norm", {"loc": 5.0, "scale": 2.0}), ("gamma", {"a": 0.7, "scale": 3.0}),
            ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}), ("poisson", {"mu": 30.0}),
            ("uniform", {}), ("expon", {}), ("lognorm", {"s": 0.5})]
    print(json.dumps(bench.ppf_sweep(_lib.load(), base, a.rows, 0), indent=1))


if __name__ == "__main__":
    main()
