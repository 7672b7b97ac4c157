"""Side measurements for BASELINE.json's other configurations (bench.py measures cfg3 only):

    cfg2  d=8 cfg2 distributions, N=1e7, native LHS fused into the inverse CDFs, no correlation
    cfg5  the README mutual-fund loop (r = r * norm(1.11, 0.15) + 1200, 20 years), N=1e8,
          scrambled Sobol', gc_strategy None (every node kept) and [] (sink only)

Each is timed through the public DAG API (`sample_device`, outputs left in HBM) with a CPU leg:
the oracle's restatement of the reference path (scipy engines + scipy ppf + numpy transforms) on a
bounded sample of the same workload.  Prints one JSON object.

    python tools/bench_configs.py [--steps 3]
"""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0


def timed(fn, steps, sync):
    fn(0)
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        fn(i + 1)
    sync()
    return (time.perf_counter() - t0) / steps


def kernel_ms(lib, calls):
    """Device time per call of each timed kernel (HIP events, pbh_timing_*) since the reset."""
    import ctypes

    from probabilit_amd import _lib

    out = {}
    for kid, name in enumerate(_lib.KERNELS):
        t, c = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(t), ctypes.byref(c)))
        if c.value:
            out[name] = {"ms_per_call": round(t.value / calls, 3), "launches_per_call": c.value / calls}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-n", type=int, default=1_000_000)
    args = ap.parse_args()
    import warnings

    import numpy as np
    import scipy.stats
    import torch

    from oracle.pipeline import cfg_dists, lhs_quantiles, mutual_fund, ppf_columns
    from probabilit_amd import device
    from probabilit_amd.modeling import Distribution, NoOp

    warnings.filterwarnings("ignore", message=".*balance properties of Sobol.*")
    dev = device.device()

    def sync():
        torch.cuda.synchronize(dev)

    out = {}
    # ---- cfg2
    n2, d2 = 10_000_000, 8
    ds = [Distribution(name, **kw) for name, kw in cfg_dists(d2)]
    root = NoOp(*ds)
    t = timed(lambda i: root.sample_device(n2, random_state=i, method="lhs"), args.steps, sync)
    t0 = time.perf_counter()
    ppf_columns(lhs_quantiles(args.cpu_n, d2, 0), cfg_dists(d2))
    tc = time.perf_counter() - t0
    out["cfg2"] = {"workload": "d=8 cfg2 set, N=1e7, native LHS + ppf", "ms": round(t * 1e3, 3),
                   "Msamples_per_s": round(n2 * d2 / t / 1e6, 1),
                   "hbm_GBps": round(8 * n2 * d2 / t / 1e9, 1), "bytes_per_draw": 8,
                   "cpu": {"Msamples_per_s": round(args.cpu_n * d2 / tc / 1e6, 3), "cores": 1, "kind": "port",
                           "sample": f"scipy LatinHypercube + scipy ppf, N={args.cpu_n}"}}

    # ---- cfg5
    n5, years = 100_000_000, 20

    def fund():
        r = 0
        for _ in range(years):
            r = r * Distribution("norm", loc=1.11, scale=0.15) + 1200
        return r

    # With 30-bit scrambled Sobol' and N >= 2^26, every 1-D projection holds one point in
    # [0, 2^-26), which is exactly 0.0 with probability 1/16 per dimension: norm.ppf(0) = -inf and
    # the reference raises ValueError (modeling.py:603-606) for most seeds.  Time seeds that pass.
    good = []
    probe = fund()
    for seed in range(200):
        try:
            probe.sample_device(n5, random_state=seed, method="sobol", gc_strategy=[])
            good.append(seed)
        except ValueError:
            pass
        if len(good) == args.steps + 1:
            break
    sync()
    out["cfg5_seeds"] = good
    from probabilit_amd import _lib, dag

    lib = _lib.load()
    for gc, label, per_row in [(None, "gc_none", 8 * (3 * years)), ([], "gc_sink", 8)]:
        sink = fund()
        fused0 = dag.counts["fused"]
        lib.pbh_timing_reset()
        lib.pbh_timing_enable(1)
        t = timed(lambda i: sink.sample_device(n5, random_state=good[i], method="sobol", gc_strategy=gc),
                  args.steps, sync)
        lib.pbh_timing_enable(0)
        calls = args.steps + 1
        out[f"cfg5_{label}"] = {"workload": f"20-step mutual fund, Sobol, N=1e8, gc_strategy={gc}",
                                "ms": round(t * 1e3, 3), "Msamples_per_s": round(n5 * years / t / 1e6, 1),
                                "hbm_GBps_retained_writes": round(per_row * n5 / t / 1e9, 1),
                                "retained_bytes_per_row": per_row,
                                "fused_calls": dag.counts["fused"] - fused0,
                                "kernels": kernel_ms(lib, calls)}
    Q = scipy.stats.qmc.Sobol(d=years, rng=0).random(args.cpu_n)
    t0 = time.perf_counter()
    mutual_fund(Q, years)
    tc = time.perf_counter() - t0
    out["cfg5_cpu"] = {"Msamples_per_s": round(args.cpu_n * years / tc / 1e6, 3), "cores": 1, "kind": "port",
                       "sample": f"scipy Sobol + scipy norm.ppf + numpy transforms, N={args.cpu_n} (engine excluded)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
