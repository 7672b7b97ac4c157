"""PermutationCorrelator restated in numpy (TEST INFRASTRUCTURE ONLY).

Follows the reference's randomized hill climb (correlation.py:473-703) and its helpers
SwapIndexGenerator (:428-470) and CorrelationMatrix (:757-921) on the same numpy calls, so that
on the same input and seed it reproduces the reference's output, printed lines and rng state
bit for bit (pinned by tests/golden/permcorr.npz).  `climb` is the hill-climbing loop alone,
from an explicit initial state: the GPU tests feed the device loop the very same state and swap
lists and require identical results.
"""

import numpy as np
import scipy.stats


def subiters(n, i):
    """Swaps per iteration i of n (correlation.py:596-608): ceil((log2 n + 1) ** (1 - 2 i / n))."""
    base = np.log2(n) + 1
    return int(np.ceil(base ** (1 - (2 * i / n))))


class SwapStream:
    """Disjoint index pairs drawn from a running permutation of range(n) (correlation.py:449-470):
    each call takes the next 2 * size entries; when fewer remain, the rest is dropped and a
    fresh permutation is drawn from the same rng."""

    def __init__(self, rng, n):
        assert n >= 2
        self.rng = rng
        self.n = n
        self.perm = rng.permutation(np.arange(n))

    def __call__(self, size):
        size = min(size, self.n // 2)
        while True:
            head, self.perm = self.perm[: 2 * size], self.perm[2 * size:]
            if len(head) == 2 * size:
                return head[:size], head[size:]
            self.perm = self.rng.permutation(np.arange(self.n))


def initial_state(X, correlation_type="pearson"):
    """CorrelationMatrix.__init__ (correlation.py:819-852): the measured space X_ (X itself, or
    its column ranks for spearman), numerator, denominator and the correlation matrix."""
    X = np.array(X, dtype=float, copy=True)
    Xs = X if correlation_type == "pearson" else np.apply_along_axis(scipy.stats.rankdata, 0, X)
    m = Xs.shape[0]
    Xc = Xs - np.mean(Xs, axis=0)
    num = (Xc.T @ Xc) / m
    den = np.std(Xc, axis=0)
    if np.any(np.isclose(den, 0)):
        raise ValueError("X has one or several constant columns")
    corr = (num / den[None, :]) / den[:, None]
    return X, Xs, num, den, corr


def delta_numerator(Xs, col, i, j):
    """Change of sum_r x_r y_r for every column when X_[i, col] and X_[j, col] swap (:875-897)."""
    ri, rj = Xs[i, :], Xs[j, :]
    d = np.sum((ri - rj) * (rj[:, col] - ri[:, col])[:, None], axis=0)
    d[col] = 0.0
    return d


def triu_error(corr, C, Wn):
    """_error (correlation.py:582-586): sqrt(sum_{a<b} w_ab (corr_ab - C_ab)^2)."""
    a, b = np.triu_indices(C.shape[0], k=1)
    return float(np.sqrt(np.sum(Wn[a, b] * (corr[a, b] - C[a, b]) ** 2.0)))


def climb(X, Xs, corr, den, C, Wn, iterations, tol, swaps, verbose_every=None):
    """The (iteration, variable) loop of __call__ (correlation.py:650-700).  `swaps(iteration)`
    returns the (i, j) index arrays of that step.  Mutates corr / Xs / X in place and returns
    (X, printed lines, steps run)."""
    m, k = Xs.shape
    lines = []
    err = triu_error(corr, C, Wn)
    it = 1
    steps = 0
    while iterations == 0 or it <= iterations:
        for col in range(k):
            if verbose_every and col == 0 and it % verbose_every == 0:
                lines.append(f" Iter {it:>6}  Error: {err:.6f} Swaps: {swaps.size_of(it):>2}")
            i, j = swaps(it)
            steps += 1
            dcol = delta_numerator(Xs, col, i, j) / (m * den * den[col])
            new = corr[:, col] + dcol
            old = corr[col, :]
            w = Wn[col, :]
            e_old = np.average((C[col, :] - old) ** 2, weights=w)
            e_new = np.average((C[col, :] - new) ** 2, weights=w)
            if e_new < e_old:
                corr[:, col] += dcol
                corr[col, :] += dcol
                Xs[i, col], Xs[j, col] = Xs[j, col], Xs[i, col]
                if Xs is not X:
                    X[i, col], X[j, col] = X[j, col], X[i, col]
            if col == 0:
                err = triu_error(corr, C, Wn)
                if err < tol:
                    if verbose_every is not None:
                        lines.append(f" Terminating at iteration {it} due to tolerance. Error: {err:.6f}")
                    return X, lines, steps
        it += 1
    return X, lines, steps


class ReferenceSwaps:
    """swaps(iteration) as the reference draws them: subiters sizes from one SwapStream."""

    def __init__(self, rng, n, iterations):
        self.stream = SwapStream(rng, n)
        self.n_sched = iterations if iterations else 10_000
        self.log = []

    def size_of(self, it):
        return subiters(self.n_sched, it)

    def __call__(self, it):
        i, j = self.stream(self.size_of(it))
        self.log.append((i, j))
        return i, j


def permutation_correlate(X, C, weights=None, iterations=1000, tol=0.01, correlation_type="pearson", seed=None,
                          verbose=False, rng=None):
    """PermutationCorrelator(...).set_target(C, weights=weights)(X): returns (Y, stdout text, rng)."""
    rng = np.random.default_rng(seed) if rng is None else rng
    W = np.ones_like(C) if weights is None else weights
    Wn = W / np.sum(W)
    n = X.shape[0]
    Xo, Xs, _, den, corr = initial_state(X, correlation_type)
    swaps = ReferenceSwaps(rng, n, iterations)
    if 0 < iterations < 10:
        raise ZeroDivisionError("integer modulo by zero")  # iteration % (iterations // 10), :660
    # iterations == 0: print_iter is the constant 1000, so no per-iteration lines (:660)
    every = (iterations // 10 if iterations else 0) if verbose else None
    Y, lines, _ = climb(Xo, Xs, corr, den, C, Wn, iterations, tol, swaps, verbose_every=every)
    head = f"Running permutation correlator for {iterations if iterations else 'inf'} iterations.\n"
    text = (head + "".join(s + "\n" for s in lines)) if verbose else ""
    return Y, text, rng
