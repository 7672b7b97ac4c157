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
    ap.add_argument("--scores", choices=("device", "reference"), default="device",
                    help="reference: the reference's own step 1 (scipy ppf, rankdata, ndtri) and step 2 too")
    a = ap.parse_args()

    import scale_parity as sp
    from oracle.pipeline import cfg3_corr

    t0 = time.time()

    def log(msg):
        print(f"[{time.time() - t0:7.1f}s] {msg if isinstance(msg, str) else json.dumps(msg)}", flush=True)

    doc = sp.gate_all(a.rows, a.d, a.seed, cfg3_corr(a.d), threads=a.threads, log=log, scores=a.scores)
    s = json.dumps(doc, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    return 0 if doc["violations_total"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
