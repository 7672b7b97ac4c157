"""CPU stand-in for probabilit_amd.distributed.HipPhases (TEST INFRASTRUCTURE ONLY).

The row-sharded Iman-Conover orchestrator (probabilit_amd/distributed.py) moves data
between ranks with torch.distributed; its compute goes through a `phases` object.  These
numpy phases implement the same contracts for an explicit LHS design (per column: a
permutation and a jitter, as scipy's LatinHypercube would give), so that world-size-2 gloo
runs on a machine without a GPU exercise every exchange: the run-head all-gather, the
column-sum and Gram all-reduces and both all-to-alls.  The expected result is the oracle's
single-process ImanConover (oracle/ic.py) on the same design.
"""

import numpy as np
import scipy.linalg
import scipy.special
import scipy.stats
import torch

from oracle.ic import rankdata_average

_NAMES = {0: "norm", 1: "uniform", 2: "expon", 3: "lognorm", 4: "triang", 5: "gamma", 6: "poisson"}
_ARGS = {"norm": ("loc", "scale"), "uniform": ("loc", "scale"), "expon": ("loc", "scale"),
         "lognorm": ("s", "loc", "scale"), "triang": ("c", "loc", "scale"), "gamma": ("a", "loc", "scale"),
         "poisson": ("mu", "loc")}


def design(n, k, seed):
    """perm[c][r] (0-based stratum of row r) and jitter u[c][r] of a k-column LHS design."""
    rng = np.random.default_rng(seed)
    perms = [rng.permutation(n) for _ in range(k)]
    us = [rng.random(n) for _ in range(k)]
    return perms, us


def column_values(col, perms, us, n):
    """X[:, c] in row order for the design (what the single-process reference sees)."""
    p, u = perms[col.lhs_col], us[col.lhs_col]
    q = (p + 1 - u) / n
    return _ppf(col, q)


def _ppf(col, q):
    name = _NAMES[col.dist]
    kw = dict(zip(_ARGS[name], col.params))
    return getattr(scipy.stats, name)(**kw).ppf(q)


class CpuPhases:
    def __init__(self, perms, us):
        self.perms = perms
        self.us = us
        self.inv = [np.argsort(p) for p in perms]

    def empty(self, shape, dtype="float64"):
        return torch.empty(shape, dtype=getattr(torch, dtype))

    def sorted_segment(self, col, n, t0, nt, flag):
        t = np.arange(t0, t0 + nt)
        rows = self.inv[col.lhs_col][t]
        q = (t + 1 - self.us[col.lhs_col][rows]) / n
        x = _ppf(col, q)
        if not np.isfinite(x).all():
            flag |= 1  # the kernels' atomicOr of bit 0
        return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64))

    def sorted_check(self, x):
        a = x.numpy()
        return int((a[:-1] == a[1:]).sum()), int((~(a[:-1] <= a[1:])).sum())

    def run_heads(self, x, t0, first_is_prev):
        a = x.numpy()
        if first_is_prev:
            h = np.flatnonzero(a[1:] != a[:-1]) + t0
        else:
            h = np.concatenate([[0], np.flatnonzero(a[1:] != a[:-1]) + 1]) + t0
        return torch.from_numpy(h.astype(np.int32))

    def scores(self, col, n, row0, nrows, heads, out):
        t = self.perms[col.lhs_col][row0:row0 + nrows]
        if heads is None:
            rank = t + 1.0
        else:
            h = heads.numpy().astype(np.int64)
            i = np.searchsorted(h, t, side="right") - 1
            s = h[i]
            e = np.append(h, n)[i + 1] - 1
            rank = (s + 1).astype(float) + (e - s) / 2.0
        out.copy_(torch.from_numpy(scipy.special.ndtri(rank / (n + 1))))

    def column_sums(self, S):
        return torch.from_numpy(S.numpy().sum(axis=1))

    def centered_gram(self, S, means):
        D = S.numpy() - means.numpy()[:, None]
        return torch.from_numpy(D @ D.T)

    def factor(self, gram, n):
        G = gram / (n - 1)
        sd = np.sqrt(np.diag(G))
        E = np.clip(G / sd[:, None] / sd[None, :], -1, 1)
        try:
            L = np.linalg.cholesky(E)
        except np.linalg.LinAlgError as err:
            raise ValueError("Rank data correlation not positive definite.") from err
        return E, L

    def apply(self, S, L, P):
        D = scipy.linalg.solve_triangular(L, S.numpy(), lower=True)
        S.copy_(torch.from_numpy(np.tril(P) @ D))

    def reorder(self, cs, sorted_src, out):
        idx = rankdata_average(cs.numpy()).astype(int) - 1
        out.copy_(torch.from_numpy(sorted_src.numpy()[idx]))
