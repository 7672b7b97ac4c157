"""§8(d) parity gate at the bench size, all columns:

    python tools/parity_1e8.py [--rows 100000000] [--d 32] [--seed 0] [--threads 8] [--out FILE]

Runs the production Iman-Conover path of the cfg3 bench workload on the GPU (natively
generated LHS columns, code-bucket step 4, LDS placement) keeping the step-1 scores S, then on
the host recomputes everything after step 1 the reference's way from those scores:
E = np.corrcoef(S) (correlation.py:398), L = np.linalg.cholesky(E) (:405),
D = scipy.linalg.solve_triangular(L, S.T, lower=True).T (:409-411), CS = D @ P.T (:414),
idx = rankdata(CS[:, k]).astype(int) - 1 (:422), and counts, per column, the rows whose
device output differs from sort(X[:, k])[idx] -- each must be one side of an adjacent-rank
swap with reference |dCS| < 1e-13.  Prints one JSON document (and writes --out).
"""

import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default="")
    a = ap.parse_args()

    import numpy as np

    import scale_parity as sp
    from oracle.pipeline import cfg3_corr
    from probabilit_amd import device

    t0 = time.time()

    def log(msg):
        print(f"[{time.time() - t0:7.1f}s] {msg}", flush=True)

    n, d = a.rows, a.d
    Y, S, CS, E_dev, P, gen = sp.run_device(n, d, a.seed, cfg3_corr(d))
    log("device run done")
    S_host = device.to_host(S)
    del S
    log("S downloaded")
    E_ref = np.corrcoef(S_host.T, rowvar=False)  # the reference's S is (N, K): S_host.T
    log(f"np.corrcoef done; max |E_dev - E_ref| = {float(np.max(np.abs(E_dev - E_ref))):.3e}")
    cs_ref = sp.reference_cs(S_host, E_ref, P)
    del S_host
    log("reference CS done")

    def one(j):
        y = device.to_host(Y[j])
        csd = device.to_host(CS[j])
        r = sp.column_gate(j, np.ascontiguousarray(cs_ref[:, j]), y, sp.sorted_x(gen[j], n), csd)
        r["max_abs_cs_dev_minus_ref"] = float(np.max(np.abs(csd - cs_ref[:, j])))
        log(json.dumps(r))
        return r

    with ThreadPoolExecutor(a.threads) as ex:
        cols = list(ex.map(one, range(d)))
    doc = {"what": "SURVEY.md §8(d) step-4 parity gate: device (production path) vs the reference's "
                   "corrcoef/cholesky/solve_triangular/@P.T/rankdata on the device scores S",
           "workload": f"cfg3 (cfg2 set x4), N={n}, d={d}, native LHS seed {a.seed}, target C = 0.9 corrcoef(A) + 0.1 I",
           "rows": n, "d": d, "seed": a.seed,
           "max_abs_E_dev_minus_ref": float(np.max(np.abs(E_dev - E_ref))),
           "mismatched_rows_total": sum(c["mismatched_rows"] for c in cols),
           "swaps_total": sum(c["swaps"] for c in cols),
           "ties_total": sum(c["ties"] for c in cols),
           "violations_total": sum(c["violations"] for c in cols),
           "max_abs_dcs_ref_in_swaps": max(c["max_abs_dcs_ref"] for c in cols),
           "max_abs_cs_dev_minus_ref": max(c["max_abs_cs_dev_minus_ref"] for c in cols),
           "seconds": round(time.time() - t0, 1), "columns": cols}
    s = json.dumps(doc, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    return 0 if doc["violations_total"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
