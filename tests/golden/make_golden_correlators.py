"""Golden fixtures for the Cholesky correlator, decorrelate and the exact pseudo-random /
Halton streams, produced by the REAL reference (stub-imported as in make_golden.py; build
container only).  Writes tests/golden/correlators.npz.

    python tests/golden/make_golden_correlators.py
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import correlation, modeling  # noqa: E402  (reference, stub-imported)


def main():
    out = {}
    rng = np.random.default_rng(2025)
    for n, k in [(9, 2), (500, 3), (2000, 8)]:
        X = rng.gamma(2.0, size=(n, k)) + rng.normal(size=(n, 1))
        A = rng.normal(size=(3 * k, k))
        C = 0.8 * np.corrcoef(A, rowvar=False) + 0.2 * np.eye(k)
        out[f"chol_X_{n}x{k}"] = X
        out[f"chol_C_{n}x{k}"] = C
        out[f"chol_Y_{n}x{k}"] = correlation.Cholesky().set_target(C)(X)
        out[f"decor_Y_{n}x{k}"] = correlation.decorrelate(X)
        out[f"decor_keepvar_Y_{n}x{k}"] = correlation.decorrelate(X, remove_variance=False)
    # Node.sample with method=None (RandomState MT19937) and method="halton", no correlation
    a = modeling.Distribution("norm", loc=1.0, scale=2.0)
    b = modeling.Distribution("expon", scale=3.0)
    expr = a * b + 1.0
    out["dag_none_s0_n1000"] = expr.sample(1000, random_state=0)
    out["dag_halton_s4_n513"] = expr.sample(513, random_state=4, method="halton")
    out["dag_none_rs_n100"] = expr.sample(100, random_state=np.random.RandomState(3))
    out["dag_none_gen_n100"] = expr.sample(100, random_state=np.random.default_rng(3))
    np.savez_compressed(os.path.join(HERE, "correlators.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
