"""Host helpers (utils.py of the reference; only what the sampling path needs)."""

import numpy as np


def build_corrmat(correlations):
    """Embed per-`correlate()` blocks into one identity-initialised K x K matrix
    (utils.py:93-115).  Unspecified pairs are 0, as in the reference.

    >>> build_corrmat([((0, 2), np.array([[1, 0.5], [0.5, 1]]))])
    array([[1. , 0. , 0.5],
           [0. , 1. , 0. ],
           [0.5, 0. , 1. ]])
    """
    k = 1 + max(max(idx) for (idx, _) in correlations)
    C = np.eye(k, dtype=float)
    for idx, block in correlations:
        C[np.ix_(idx, idx)] = block
    return C
