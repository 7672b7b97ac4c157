"""Iman-Conover restated in numpy (TEST INFRASTRUCTURE ONLY).

Follows ImanConover.__call__ (correlation.py:368-425) step by step and returns every
intermediate.  rankdata('average') is restated from scipy:stats/_stats_py.py _rankdata:
quicksort argsort, run heads where sorted neighbours differ, rank = ordinal(head) +
(count - 1) / 2, scattered back through the argsort.

`threads` spreads the per-column work (the two rankdata passes, the ndtri of the scores,
the sorted-X gather) over a thread pool for the large parity cases (numpy's sorts and
ufunc loops release the GIL).  Every column is computed by exactly the same numpy calls as
in the sequential form, so the results are identical bit for bit; the matrix steps
(corrcoef, cholesky, solve_triangular, matmul) are single calls either way.
"""

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import scipy.linalg
import scipy.special


def rankdata_average(x):
    x = np.asarray(x, dtype=float)
    n = x.shape[0]
    j = np.argsort(x, kind="quicksort")
    y = x[j]
    head = np.concatenate([[True], y[:-1] != y[1:]])
    starts = np.flatnonzero(head)
    counts = np.diff(np.append(starts, n))
    ranks_sorted = np.repeat((starts + 1) + (counts - 1) / 2, counts)
    out = np.empty(n)
    out[j] = ranks_sorted
    return out


def _map(fn, items, threads):
    if not threads or threads <= 1:
        return [fn(i) for i in items]
    with ThreadPoolExecutor(threads) as ex:
        return list(ex.map(fn, items))


def iman_conover(X, C, threads=None):
    """Returns dict(Y, S, E, L, CS, idx) for data X (N, K) and target correlation C."""
    X = np.asarray(X, dtype=float)
    N, K = X.shape
    P = np.linalg.cholesky(C)
    ranks = np.empty((N, K))
    S = np.empty((N, K))

    def step1(k):
        ranks[:, k] = rankdata_average(X[:, k]) / (N + 1)                              # :394
        S[:, k] = scipy.special.ndtri(ranks[:, k])                                     # :395

    _map(step1, range(K), threads)
    E = np.corrcoef(S, rowvar=False)                                                   # :398
    L = np.linalg.cholesky(E)                                                          # :405
    D = scipy.linalg.solve_triangular(L, S.T, lower=True).T                            # :409-411
    CS = D @ P.T                                                                       # :414
    idx = np.empty((N, K), dtype=np.int64)
    Y = np.empty((N, K))

    def step4(k):
        idx[:, k] = rankdata_average(CS[:, k]).astype(int) - 1                         # :422
        Y[:, k] = np.sort(X[:, k])[idx[:, k]]                                          # :423

    _map(step4, range(K), threads)
    return {"Y": Y, "S": S, "E": E, "L": L, "CS": CS, "idx": idx}
