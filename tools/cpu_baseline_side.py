"""Side measurement of the reference's CPU path (oracle.pipeline.lhs_ic: scipy LHS -> scipy ppf
-> the reference's Iman-Conover in numpy / scipy) at the given sizes, on this host.  It is the
cpu_baseline of bench.py at more than one N (1e6 and 1e7), with the thread
settings stated; never `value`.

    python tools/cpu_baseline_side.py --rows 1000000 10000000 > profiles/r02/cpu_baseline_side.json
"""

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, nargs="+", default=[1_000_000, 10_000_000])
    ap.add_argument("--d", type=int, default=32)
    a = ap.parse_args()
    from threadpoolctl import threadpool_info

    from oracle.pipeline import lhs_ic

    import threading

    def heartbeat():  # a long CPU run must keep writing (the GPU box's watchdog kills silent runs)
        t0 = time.perf_counter()
        while True:
            time.sleep(30)
            print(f"... {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    out = []
    for n in a.rows:
        t0 = time.perf_counter()
        lhs_ic(n, a.d, 0)
        dt = time.perf_counter() - t0
        rate = n * a.d / dt / 1e6
        out.append({"rows": n, "d": a.d, "seconds": round(dt, 2), "Msamples_per_s": round(rate, 4),
                    "nlogn_extrapolated_1e8": round(rate * math.log(n) / math.log(1e8), 4)})
        print(json.dumps(out[-1]), file=sys.stderr, flush=True)
    threads = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    print(json.dumps({"what": "oracle.pipeline.lhs_ic (cfg3 set, LHS + ppf + Iman-Conover), CPU", "runs": out,
                      "blas_threads": threads, "nproc": os.cpu_count(),
                      "openblas_num_threads": os.environ.get("OPENBLAS_NUM_THREADS"),
                      "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
                      "note": "ppf and sorts single-threaded (scipy / numpy); BLAS pool as stated"}, indent=1))


if __name__ == "__main__":
    main()
