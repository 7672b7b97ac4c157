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
    """redo: owned column indices whose first ranking is "rejected" (garbage positions leave
    first, the correct ones after owned_finish), to exercise the re-send of a redone column."""

    def __init__(self, perms, us, redo=(), fake_tie=None):
        self.perms = perms
        self.us = us
        self.inv = [np.argsort(p) for p in perms]
        self.redo = set(redo)
        self.fake_tie = fake_tie  # column whose first count reports a (false) tie: the deferred check redoes

    def empty(self, shape, dtype="float64"):
        return torch.empty(shape, dtype=getattr(torch, dtype))

    def zeros(self, shape, dtype="float64"):
        return torch.zeros(shape, dtype=getattr(torch, dtype))

    def _sorted(self, col, n, t):
        rows = self.inv[col.lhs_col][t]
        q = (t + 1 - self.us[col.lhs_col][rows]) / n
        return _ppf(col, q)

    # -- step 1
    def sorted_counts(self, col, n, t0, nt, flag, counts, heads=None, hcur=None, certify=False):
        x = self._sorted(col, n, np.arange(t0, t0 + nt))
        if not np.isfinite(x).all():
            flag |= 1  # the kernels' atomicOr of bit 0
        counts[0] = int((x[:-1] == x[1:]).sum())
        counts[1] = int((~(x[:-1] <= x[1:])).sum())
        if self.fake_tie == col.lhs_col:
            counts[0] += 1
            self.fake_tie = None
        if heads is not None:
            h = np.flatnonzero(x[1:] != x[:-1]) + t0 + 1
            if t0 == 0:
                h = np.concatenate([[0], h])
            h = h[::-1]  # appended out of order, as the kernel's atomics do
            cap = heads.shape[0]
            heads[:min(len(h), cap)] = torch.from_numpy(h[:cap].astype(np.int32))
            hcur[0] = len(h)

    def sort_heads(self, heads):
        heads.copy_(torch.sort(heads).values)

    def segment_heads(self, col, n, t0, nt, first_is_prev, flag):
        a = self._sorted(col, n, np.arange(t0, t0 + nt))
        if first_is_prev:
            h = np.flatnonzero(a[1:] != a[:-1]) + t0 + 1
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

    # -- steps 2 and 3
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

    # -- step 4 (synchronous: no events)
    def ready(self, owned):
        return None

    def wait(self, ev, stream=None):
        pass

    def owned_begin(self, cols, n):
        return {"cols": cols, "n": n, "pending": {}}

    def owned_column(self, owned, i, cs, p_out, ready):
        idx = rankdata_average(cs.numpy()).astype(int) - 1
        if i in self.redo:
            owned["pending"][i] = (p_out, idx)
            p_out.fill_(0)  # what leaves first: wrong
        else:
            p_out.copy_(torch.from_numpy(idx.astype(np.int32)))
        return None

    def owned_finish(self, owned):
        for p_out, idx in owned["pending"].values():
            p_out.copy_(torch.from_numpy(idx.astype(np.int32)))
        return sorted(owned["pending"])

    def owned_end(self, owned):
        pass

    def values_at(self, col, n, p, y):
        y.copy_(torch.from_numpy(self._sorted(col, n, p.numpy().astype(np.int64))))

    # -- materialised columns on their owner (distributed.iman_conover_block)
    def column_scores(self, x, s_out, sx_out, flag):
        xv = x.numpy().copy()  # s_out may be x itself
        if np.isnan(xv).any():
            flag |= 1
        r = rankdata_average(xv)
        sx_out.copy_(torch.from_numpy(np.sort(xv)))
        s_out.copy_(torch.from_numpy(scipy.special.ndtri(r / (len(xv) + 1))))

    def reorder(self, cs, sx, y):
        idx = rankdata_average(cs.numpy()).astype(int) - 1
        y.copy_(torch.from_numpy(sx.numpy()[idx]))
