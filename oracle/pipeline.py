"""BASELINE.json configurations on the CPU, the way the reference computes them
(TEST INFRASTRUCTURE ONLY; the cpu_baseline leg of bench.py times these).

cfg2/cfg3: LatinHypercube quantiles (modeling.py:480,488) -> scipy ppf per column
(modeling.py:807) -> Iman-Conover (correlation.py:368-425, restated in oracle.ic).
cfg5: the README mutual-fund chain r = r * norm(1.11, 0.15) + 1200 over 20 years.
"""

import numpy as np
import scipy.stats

from . import ic
from .ppf import ppf

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


def cfg_dists(d):
    return (CFG2 * ((d + 7) // 8))[:d]


def cfg3_corr(d=32):
    A = np.random.default_rng(0).normal(size=(64, d))
    return 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(d)


def lhs_quantiles(n, d, seed):
    return scipy.stats.qmc.LatinHypercube(d=d, rng=seed).random(n)


def ppf_columns(Q, dists, threads=None, chunk=1 << 20):
    """Column j = scipy.stats.<dist_j>(**kw).ppf(Q[:, j]) (modeling.py:807).  With `threads`,
    each column is cut into row chunks evaluated on a thread pool (the same elementwise
    scipy call per chunk, so identical values)."""
    if not threads or threads <= 1:
        return np.column_stack([ppf(name, Q[:, j], **kw) for j, (name, kw) in enumerate(dists)])
    from concurrent.futures import ThreadPoolExecutor

    n = Q.shape[0]
    out = np.empty((n, len(dists)))
    tasks = [(j, r0) for j in range(len(dists)) for r0 in range(0, n, chunk)]

    def run(t):
        j, r0 = t
        name, kw = dists[j]
        out[r0:r0 + chunk, j] = ppf(name, np.ascontiguousarray(Q[r0:r0 + chunk, j]), **kw)

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, tasks))
    return out


def lhs_ic(n, d, seed, C=None):
    """cfg3 end to end on the CPU: returns (Q, X, Y)."""
    C = cfg3_corr(d) if C is None else C
    Q = lhs_quantiles(n, d, seed)
    X = ppf_columns(Q, cfg_dists(d))
    return Q, X, ic.iman_conover(X, C)["Y"]


def mutual_fund(Q, years=20, loc=1.11, scale=0.15, saved=1200):
    r = None
    for y in range(years):
        interest = ppf("norm", Q[:, y], loc=loc, scale=scale)
        r = interest * 0 + saved if r is None else r * interest + saved
    return r
