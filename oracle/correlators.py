"""The reference's other correlators restated in numpy (TEST INFRASTRUCTURE ONLY).

cholesky_transform follows Cholesky.__call__ (correlation.py:249-285) and decorrelate follows
correlation.py:706-754, line by line, on the same numpy / scipy calls.
"""

import numpy as np
import scipy.linalg


def cholesky_transform(X, C):
    X = np.asarray(X, dtype=float)
    target_P = np.linalg.cholesky(C)
    mean = np.mean(X, axis=0)                                   # :271
    std = np.std(X, axis=0)                                     # :272
    X_n = (X - mean) / std                                      # :273
    cov = np.cov(X_n, rowvar=False, ddof=0)                     # :276
    P = np.linalg.cholesky(cov)                                 # :277
    transform = scipy.linalg.solve_triangular(P.T, target_P.T, lower=False)  # :284
    return mean + X_n @ (transform * std)                       # :285


def decorrelate(X, remove_variance=True):
    X = np.asarray(X, dtype=float)
    mean = np.mean(X, axis=0)                                   # :745
    var = np.var(X, axis=0, ddof=0)                             # :746
    cov = np.cov(X, rowvar=False)                               # :747
    L = np.linalg.cholesky(cov)                                 # :749
    if not remove_variance:
        L = L / np.sqrt(var)                                    # :751
    X = scipy.linalg.solve_triangular(L, (X - mean).T, lower=True).T  # :754
    return mean + X
