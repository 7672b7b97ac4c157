"""Generate the golden parity fixtures under tests/golden/ from the REAL reference.

Runs only in the build container, where /root/reference exists.  It imports the
reference package (tommyod/probabilit @ 2025-09-19) through empty stub modules
for `cvxpy` and `seaborn` (both absent from the image; SURVEY.md §8c recipe) and
records inputs and outputs as small .npz files.  Nothing here is imported by the
product or by the GPU tests: the .npz files are the data that travels.

Where the reference path needs cvxpy (`nearest_correlation_matrix`, called at
modeling.py:574 on every correlated `.sample()`), the generator substitutes the
identity map for an already-valid target C and records `ncm="identity"` in the
fixture metadata.

Usage:  python tests/golden/make_golden.py      (writes tests/golden/*.npz)
"""

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _import_reference():
    stub_dir = tempfile.mkdtemp(prefix="pbh_stubs_")
    for mod in ("cvxpy", "seaborn"):
        with open(os.path.join(stub_dir, mod + ".py"), "w") as fh:
            fh.write("")
    sys.path.insert(0, REF_SRC)
    sys.path.insert(0, stub_dir)
    sys.dont_write_bytecode = True
    import probabilit  # noqa: F401
    import probabilit.modeling as modeling
    import probabilit.correlation as correlation

    return modeling, correlation


modeling, correlation = _import_reference()
import scipy as sp  # noqa: E402
from scipy import stats  # noqa: E402


# ---------------------------------------------------------------------------
# distribution sets of BASELINE.json configs 2/3 (creation order matters)
# ---------------------------------------------------------------------------
CFG2 = [
    ("norm", {"loc": 0.0, "scale": 1.0}),
    ("gamma", {"a": 2.0}),
    ("triang", {"c": 0.3}),
    ("poisson", {"mu": 4.0}),
    ("norm", {"loc": 5.0, "scale": 2.0}),
    ("gamma", {"a": 0.7, "scale": 3.0}),
    ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}),
    ("poisson", {"mu": 30.0}),
]


def cfg3_corr(d=32):
    A = np.random.default_rng(0).normal(size=(64, d))
    return 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(d)


def ppf(name, q, kw):
    return getattr(stats, name)(**kw).ppf(q)


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


# ---------------------------------------------------------------------------
# G1: quantile streams
# ---------------------------------------------------------------------------
def gen_streams():
    out = {}
    eng = stats.qmc.LatinHypercube(d=8, rng=0)
    st = eng.rng.bit_generator.state
    out["lhs_d8_s0_state"] = np.array(
        [st["state"]["state"] >> 64, st["state"]["state"] & (2**64 - 1),
         st["state"]["inc"] >> 64, st["state"]["inc"] & (2**64 - 1)], dtype=np.uint64)
    out["lhs_d8_s0_n4096"] = eng.random(4096)
    eng = stats.qmc.LatinHypercube(d=3, rng=123)
    out["lhs_d3_s123_n1000"] = eng.random(1000)

    for d, seed, n in ((20, 0, 4096), (5, 7, 1000), (32, 1, 512)):
        eng = stats.qmc.Sobol(d=d, rng=seed)
        out[f"sobol_d{d}_s{seed}_sv"] = eng._sv.copy()
        out[f"sobol_d{d}_s{seed}_shift"] = eng._shift.copy()
        with np.errstate(all="ignore"):
            import warnings

            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                out[f"sobol_d{d}_s{seed}_n{n}"] = eng.random(n)
    unscr = stats.qmc.Sobol(d=20, scramble=False)
    out["sobol_d20_unscrambled_sv"] = unscr._sv.copy()
    out["mt_s0_999x1"] = np.random.RandomState(0).random((999, 1))
    save("streams.npz", **out)


# ---------------------------------------------------------------------------
# G2: ppf (scipy.stats.<dist>.ppf, the call at modeling.py:807)
# ---------------------------------------------------------------------------
EDGE_Q = np.array([0.0, 5e-324, 1e-300, 1e-20, 2.0**-53, 1e-10, 0.001, 0.25, 0.5,
                   0.75, 0.9, 0.999, 1 - 1e-10, 1 - 2.0**-53, 1.0, np.nan, -0.1, 1.1])

PPF_CASES = {
    "norm_std": ("norm", {}),
    "norm_176": ("norm", {"loc": 176.0, "scale": 7.1}),
    "uniform": ("uniform", {"loc": -2.0, "scale": 5.0}),
    "expon": ("expon", {"scale": 1 / 3}),
    "lognorm": ("lognorm", {"s": 0.5, "scale": 2.0}),
    "triang_c0": ("triang", {"c": 0.0}),
    "triang_c03": ("triang", {"c": 0.3}),
    "triang_c08": ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}),
    "triang_c1": ("triang", {"c": 1.0}),
    "gamma_a01": ("gamma", {"a": 0.1}),
    "gamma_a07": ("gamma", {"a": 0.7, "scale": 3.0}),
    "gamma_a1": ("gamma", {"a": 1.0}),
    "gamma_a2": ("gamma", {"a": 2.0}),
    "gamma_a20": ("gamma", {"a": 20.0, "loc": -1.0}),
    "gamma_a250": ("gamma", {"a": 250.0}),
    "gamma_a3000": ("gamma", {"a": 3000.0}),
    "poisson_mu0": ("poisson", {"mu": 0.0}),
    "poisson_mu05": ("poisson", {"mu": 0.5}),
    "poisson_mu4": ("poisson", {"mu": 4.0}),
    "poisson_mu30": ("poisson", {"mu": 30.0, "loc": 2.0}),
    "poisson_mu1000": ("poisson", {"mu": 1000.0}),
    "norm_badscale": ("norm", {"scale": -1.0}),
    "gamma_bad_a": ("gamma", {"a": -1.0}),
    "poisson_bad_mu": ("poisson", {"mu": -1.0}),
}


def gen_ppf():
    q_lhs = stats.qmc.LatinHypercube(d=1, rng=5).random(4096)[:, 0]
    q = np.concatenate([q_lhs, EDGE_Q])
    out = {"q": q}
    meta = {}
    for name, (dist, kw) in PPF_CASES.items():
        with np.errstate(all="ignore"):
            out[name] = ppf(dist, q, kw)
        meta[name] = [dist, kw]
    # composite (array-valued) parameters: modeling.py:796-802 broadcast
    rng = np.random.default_rng(11)
    n = q.size
    loc = rng.normal(size=n)
    scale = rng.uniform(0.5, 2.0, size=n)
    mu = rng.uniform(0.0, 60.0, size=n)
    a = rng.uniform(0.05, 40.0, size=n)
    c = rng.uniform(0.0, 1.0, size=n)
    out["comp_loc"], out["comp_scale"], out["comp_mu"], out["comp_a"], out["comp_c"] = loc, scale, mu, a, c
    with np.errstate(all="ignore"):
        out["comp_norm"] = stats.norm(loc=loc, scale=scale).ppf(q)
        out["comp_poisson"] = stats.poisson(mu=mu).ppf(q)
        out["comp_gamma"] = stats.gamma(a=a, scale=scale).ppf(q)
        out["comp_triang"] = stats.triang(c=c, loc=loc, scale=scale).ppf(q)
    out["meta"] = np.array(json.dumps(meta))
    save("ppf.npz", **out)


# ---------------------------------------------------------------------------
# G3: Iman-Conover (correlation.py:368-425) incl. intermediates
# ---------------------------------------------------------------------------
def ic_intermediates(X, C):
    """Same numpy/scipy calls as correlation.py:388-425, keeping intermediates."""
    N, K = X.shape
    ranks = stats.rankdata(X, axis=0) / (N + 1)
    S = stats.norm.ppf(ranks)
    E = np.corrcoef(S, rowvar=False)
    L = np.linalg.cholesky(E)
    D = sp.linalg.solve_triangular(L, S.T, lower=True).T
    P = np.linalg.cholesky(C)
    CS = D @ P.T
    idx = np.empty((N, K), dtype=np.int64)
    for k in range(K):
        idx[:, k] = stats.rankdata(CS[:, k]).astype(int) - 1
    return ranks, S, E, L, CS, idx


def gen_ic():
    out = {}
    for tag, d, n in (("cfg2", 8, 4096), ("cfg3", 32, 2048)):
        dists = (CFG2 * (d // 8))[:d]
        Q = stats.qmc.LatinHypercube(d=d, rng=0).random(n)
        X = np.column_stack([ppf(nm, Q[:, j], kw) for j, (nm, kw) in enumerate(dists)])
        C = cfg3_corr(d)
        Y = correlation.ImanConover().set_target(C)(X)
        ranks, S, E, L, CS, idx = ic_intermediates(X, C)
        assert np.array_equal(Y, np.column_stack([np.sort(X[:, k])[idx[:, k]] for k in range(d)]))
        out.update({f"{tag}_X": X, f"{tag}_C": C, f"{tag}_Y": Y, f"{tag}_S": S, f"{tag}_E": E,
                    f"{tag}_L": L, f"{tag}_CS": CS, f"{tag}_idx": idx.astype(np.int32)})
    # tie quirk: discrete leading columns
    Q = stats.qmc.LatinHypercube(d=3, rng=1).random(20000)
    X = np.column_stack([stats.poisson(4).ppf(Q[:, 0]), stats.poisson(3).ppf(Q[:, 1]),
                         stats.norm().ppf(Q[:, 2])])
    C = np.array([[1, 0.5, 0.3], [0.5, 1, 0.2], [0.3, 0.2, 1.0]])
    Y = correlation.ImanConover().set_target(C)(X)
    ranks, S, E, L, CS, idx = ic_intermediates(X, C)
    out.update({"ties_X": X, "ties_C": C, "ties_Y": Y, "ties_S": S, "ties_CS": CS, "ties_idx": idx.astype(np.int32)})
    # doctest toy correlation.py:315-330
    Xt = np.array([[0, 0], [0, 0.5], [0, 1], [1, 0], [1, 0.5], [1, 1]], dtype=float)
    Ct = np.array([[1, 0.7], [0.7, 1]])
    out.update({"toy_X": Xt, "toy_C": Ct, "toy_Y": correlation.ImanConover().set_target(Ct)(Xt)})
    # normal / lognormal doctest stats correlation.py:347-361
    rng = np.random.default_rng(42)
    Xn = rng.normal(size=(1000, 2))
    out.update({"normal_X": Xn, "normal_Y": correlation.ImanConover().set_target(Ct)(Xn)})
    rng = np.random.default_rng(42)
    Xl = rng.lognormal(size=(1000, 2))
    out.update({"lognormal_X": Xl, "lognormal_Y": correlation.ImanConover().set_target(Ct)(Xl)})
    # README IC example (README.md:110-130)
    sampler = stats.qmc.LatinHypercube(d=2, seed=42, scramble=True)
    samples = sampler.random(n=100)
    Xr = np.vstack((stats.triang(0.5).ppf(samples[:, 0]), stats.gamma.ppf(samples[:, 1], a=1))).T
    Cr = np.array([[1, 0.3], [0.3, 1]])
    out.update({"readme_X": Xr, "readme_C": Cr, "readme_Y": correlation.ImanConover().set_target(Cr)(Xr)})
    # Cholesky correlator doctest correlation.py:217-237
    Xc = np.random.default_rng(4).normal(size=(9, 2))
    out.update({"chol_X": Xc, "chol_C": Ct, "chol_Y": correlation.Cholesky().set_target(Ct)(Xc)})
    save("ic.npz", **out)


# ---------------------------------------------------------------------------
# G4: DAG evaluation through Node.sample_from_quantiles (modeling.py:495-614)
# ---------------------------------------------------------------------------
def _node_samples(nodes):
    return [np.asarray(n.samples_) if getattr(n, "samples_", None) is not None else np.array([])
            for n in nodes]


def gen_dag():
    M = modeling
    out = {}
    modeling.nearest_correlation_matrix = lambda C: C  # identity NCM (valid C), see module doc

    # mutual fund (README.md:64-78, cfg5 shape): sink + every interest node
    def fund():
        nodes = []
        r = 0
        for _ in range(20):
            i = M.Distribution("norm", loc=1.11, scale=0.15)
            nodes.append(i)
            r = r * i + 1200
        return r, nodes

    r, nodes = fund()
    with np.errstate(all="ignore"):
        import warnings

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            Q = stats.qmc.Sobol(d=20, rng=0).random(4096)
    out["fund_Q"] = Q
    out["fund_sink"] = r.sample_from_quantiles(Q)
    out["fund_interest"] = np.column_stack([n.samples_ for n in nodes])
    r, nodes = fund()
    Qmt = np.random.RandomState(42).random((999, 20))
    out["fund999_Q"] = Qmt
    out["fund999_sink"] = r.sample(999, random_state=42)

    # README example 1 (pseudo-random MT19937 stream)
    male = M.Distribution("norm", loc=176, scale=7.1)
    female = M.Distribution("norm", loc=162.5, scale=7.1)
    stat = male > female
    out["height_Q"] = np.random.RandomState(0).random((999, 2))
    out["height_sink"] = stat.sample(999, random_state=0)
    out["height_male"] = male.samples_

    # column assignment: mu<-col0, b<-col1, a<-col2
    mu = M.Distribution("norm")
    a = M.Distribution("norm", loc=mu)
    b = M.Distribution("expon")
    e = a + b
    e.sample_from_quantiles(np.array([[0.1, 0.2, 0.3]]))
    out["colorder"] = np.array([mu.samples_[0], a.samples_[0], b.samples_[0], e.samples_[0]])

    # expression doctest modeling.py:59-79 structure (pow/mul/add) on fixed quantiles
    a = M.Distribution("norm", loc=5, scale=1)
    b = M.Distribution("expon", scale=1)
    expr = a ** b + a * b + 5 * b
    Qe = stats.qmc.LatinHypercube(d=2, rng=3).random(257)
    out["expr_Q"] = Qe
    out["expr_sink"] = expr.sample_from_quantiles(Qe)

    # composite parameters: poisson(mu=gamma) and norm(loc=norm, scale=triang)
    g = M.Distribution("gamma", a=2.0, scale=3.0)
    p = M.Distribution("poisson", mu=g)
    m = M.Distribution("norm", loc=5.0, scale=1.0)
    s = M.Distribution("triang", c=0.4, loc=0.5, scale=1.0)
    n2 = M.Distribution("norm", loc=m, scale=s)
    root = p + n2 * 2 - 1
    Qc = stats.qmc.LatinHypercube(d=5, rng=9).random(2000)
    out["comp_Q"] = Qc
    out["comp_sink"] = root.sample_from_quantiles(Qc)
    out["comp_nodes"] = np.column_stack([g.samples_, m.samples_, s.samples_, p.samples_, n2.samples_])

    # correlated DAG, cfg3-shaped but small: NoOp(*ds).correlate(*ds, C)
    for tag, d, n in (("corr8", 8, 3000), ("corr32", 32, 2048)):
        ds = [M.Distribution(nm, **kw) for nm, kw in (CFG2 * (d // 8))[:d]]
        C = cfg3_corr(d)
        root = M.NoOp(*ds).correlate(*ds, corr_mat=C)
        Qd = stats.qmc.LatinHypercube(d=d, rng=0).random(n)
        root.sample_from_quantiles(Qd)
        out[f"{tag}_Q"], out[f"{tag}_C"] = Qd, C
        out[f"{tag}_Y"] = np.column_stack([x.samples_ for x in ds])

    # gc_strategy=[] keeps only the sink (garbage_collector.py:42-71)
    a = M.Distribution("norm")
    inter = (a + a) ** 2 - a
    final = M.Exp(inter)
    Qg = np.array([[0.2], [0.5], [0.9]])
    out["gc_sink"] = final.sample_from_quantiles(Qg, gc_strategy=[])
    out["gc_has"] = np.array([hasattr(a, "samples_"), hasattr(inter, "samples_")])

    out["meta"] = np.array(json.dumps({"ncm": "identity", "reference": "tommyod/probabilit@2025-09-19",
                                       "numpy": np.__version__, "scipy": sp.__version__}))
    save("dag.npz", **out)


if __name__ == "__main__":
    gen_streams()
    gen_ppf()
    gen_ic()
    gen_dag()
