"""Iman-Conover restated in numpy (TEST INFRASTRUCTURE ONLY).

Follows ImanConover.__call__ (correlation.py:368-425) step by step and returns every
intermediate.  rankdata('average') is restated from scipy:stats/_stats_py.py _rankdata:
quicksort argsort, run heads where sorted neighbours differ, rank = ordinal(head) +
(count - 1) / 2, scattered back through the argsort.
"""

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


def iman_conover(X, C):
    """Returns dict(Y, S, E, L, CS, idx) for data X (N, K) and target correlation C."""
    X = np.asarray(X, dtype=float)
    N, K = X.shape
    P = np.linalg.cholesky(C)
    ranks = np.column_stack([rankdata_average(X[:, k]) for k in range(K)]) / (N + 1)   # :394
    S = scipy.special.ndtri(ranks)                                                     # :395
    E = np.corrcoef(S, rowvar=False)                                                   # :398
    L = np.linalg.cholesky(E)                                                          # :405
    D = scipy.linalg.solve_triangular(L, S.T, lower=True).T                            # :409-411
    CS = D @ P.T                                                                       # :414
    idx = np.column_stack([rankdata_average(CS[:, k]).astype(int) - 1 for k in range(K)])  # :422
    Y = np.column_stack([np.sort(X[:, k])[idx[:, k]] for k in range(K)])              # :423
    return {"Y": Y, "S": S, "E": E, "L": L, "CS": CS, "idx": idx}
