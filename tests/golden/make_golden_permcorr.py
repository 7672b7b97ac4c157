"""Golden fixtures for PermutationCorrelator / CorrelationMatrix / SwapIndexGenerator
(correlation.py:428-703, 757-921), produced by the REAL reference (stub-imported as in
make_golden.py; build container only).  Writes tests/golden/permcorr.npz.

Every case stores the input X, the target C (and weights), the constructor arguments, the
output X, the verbose text and the PCG64 state of the correlator's rng after the call (the
swap-index stream must be consumed exactly as the reference consumes it).

    python tests/golden/make_golden_permcorr.py
"""

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import correlation  # noqa: E402  (reference, stub-imported)


def _state(rng):
    st = rng.bit_generator.state
    return json.dumps({"state": str(st["state"]["state"]), "inc": str(st["state"]["inc"]),
                       "has_uint32": int(st["has_uint32"]), "uinteger": int(st["uinteger"])})


def _corr(k, seed, rho=None):
    if rho is not None:
        C = np.full((k, k), rho)
        np.fill_diagonal(C, 1.0)
        return C
    A = np.random.default_rng(seed).normal(size=(3 * k, k))
    return 0.7 * np.corrcoef(A, rowvar=False) + 0.3 * np.eye(k)


def main():
    out = {}
    meta = {}

    def run(name, X, C, kwargs, weights=None):
        pc = correlation.PermutationCorrelator(**kwargs)
        pc = pc.set_target(C, weights=weights) if weights is not None else pc.set_target(C)
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            Y = pc(X)
        out[f"{name}_X"] = X
        out[f"{name}_C"] = C
        if weights is not None:
            out[f"{name}_W"] = weights
        out[f"{name}_Y"] = Y
        meta[name] = {"kwargs": kwargs, "stdout": buf.getvalue(), "rng_after": _state(pc.rng),
                      "weights": weights is not None}

    # docstring examples (correlation.py:511-560)
    rng = np.random.default_rng(42)
    X = rng.normal(size=(100, 2))
    run("doc2", X, np.array([[1, 0.7], [0.7, 1]]), {"seed": 0})
    variables = 25
    C25 = _corr(variables, 0, rho=0.7)
    X = rng.normal(size=(10 * variables, variables))
    X_ic = correlation.ImanConover().set_target(C25)(X)
    run("doc25", X_ic, C25, {"iterations": 250, "tol": 1e-6, "seed": 0, "verbose": True})

    g = np.random.default_rng(7)
    cases = [
        ("p_50x3", 50, 3, {"iterations": 40, "tol": 1e-9, "seed": 1}, False),
        ("p_1000x8", 1000, 8, {"iterations": 120, "tol": 1e-9, "seed": 2}, False),
        ("p_3000x32", 3000, 32, {"iterations": 60, "tol": 1e-9, "seed": 3, "verbose": True}, False),
        ("s_400x5", 400, 5, {"iterations": 80, "tol": 1e-9, "seed": 4, "correlation_type": "spearman"}, True),
        ("s_2000x12", 2000, 12, {"iterations": 50, "tol": 1e-9, "seed": 5, "correlation_type": "spearman",
                                 "verbose": True}, True),
        ("tol_300x4", 300, 4, {"iterations": 500, "tol": 0.02, "seed": 6}, False),
        ("inf_200x3", 200, 3, {"iterations": 0, "tol": 0.03, "seed": 8}, False),
        ("odd_7x3", 7, 3, {"iterations": 30, "tol": 1e-9, "seed": 9}, False),
        ("w_600x6", 600, 6, {"iterations": 70, "tol": 1e-9, "seed": 10}, False),
    ]
    for name, n, k, kw, ties in cases:
        X = g.gamma(2.0, size=(n, k)) + g.normal(size=(n, 1))
        if ties:  # integer-valued columns: rankdata ties in the spearman space
            X[:, 0] = g.poisson(3.0, size=n)
            X[:, 1] = np.round(X[:, 1], 1)
        W = None
        if name.startswith("w_"):
            W = g.uniform(0.5, 2.0, size=(k, k))
            W = (W + W.T) / 2
        run(name, X, _corr(k, k), kw, weights=W)

    # SwapIndexGenerator stream (correlation.py:428-470): sizes through an exhaustion
    sg = correlation.SwapIndexGenerator(rng=np.random.default_rng(11), n=9)
    sizes = [2, 2, 1, 10, 3, 1, 4, 4, 2, 1]
    flat = []
    for s in sizes:
        a, b = sg(s)
        flat.append(np.concatenate([a, b]))
    out["swapgen_n9_sizes"] = np.array(sizes)
    out["swapgen_n9_flat"] = np.concatenate(flat)
    out["swapgen_n9_lens"] = np.array([len(f) for f in flat])
    meta["subiters"] = {str(n): [correlation.PermutationCorrelator.subiters(n, i) for i in range(1, n + 1)]
                        for n in (2, 8, 250, 1000, 10000)}

    # CorrelationMatrix docstring (correlation.py:779-817) + a spearman case
    rng = np.random.default_rng(42)
    X = rng.normal(size=(9, 4))
    cm = correlation.CorrelationMatrix(X)
    out["cm_X"] = X
    out["cm_corr0"] = cm[:, :].copy()
    out["cm_update_0_2_3"] = cm.update_column(col=0, i=2, j=3)
    out["cm_update_0_01_23"] = cm.update_column(col=0, i=[0, 1], j=[2, 3])
    cm.commit(col=1, i=[4, 5], j=[6, 8])
    out["cm_after_commit"] = cm[:, :].copy()
    out["cm_X_after_commit"] = cm.X.copy()
    Xs = np.round(np.random.default_rng(3).normal(size=(30, 3)), 1)
    cms = correlation.CorrelationMatrix(Xs, correlation_type="spearman")
    out["cms_X"] = Xs
    out["cms_corr0"] = cms[:, :].copy()
    cms.commit(col=2, i=[0, 7], j=[3, 29])
    out["cms_after_commit"] = cms[:, :].copy()
    out["cms_X_after_commit"] = cms.X.copy()

    out["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, "permcorr.npz"), **out)
    print({k: getattr(v, "shape", None) for k, v in out.items()})


if __name__ == "__main__":
    main()
