"""Inverse CDF as the reference computes it (TEST INFRASTRUCTURE ONLY).

Distribution._sample (modeling.py:795-807) is `getattr(scipy.stats, name)(*args, **kw).ppf(q)`;
the oracle makes the same call on scipy 1.15.3 (the reference's pinned L0 dependency, present
here and on the GPU box).  tests/test_oracle.py pins it to tests/golden/ppf.npz, which the
reference produced.
"""

import numpy as np
import scipy.stats


def ppf(name, q, **params):
    with np.errstate(all="ignore"):
        return getattr(scipy.stats, name)(**params).ppf(q)


def poisson_smallest_k(q, mu):
    """Definition used by the device kernel: smallest k >= 0 with pdtr(k, mu) >= q
    (equivalent to scipy's ceil(pdtrik) + one-step pdtr correction on the tested range)."""
    import scipy.special as sc

    q = np.asarray(q, dtype=float)
    out = np.empty_like(q)
    for i, qi in np.ndenumerate(q):
        k = max(0.0, np.floor(mu + np.sqrt(mu) * sc.ndtri(qi)))
        if sc.pdtr(k, mu) >= qi:
            while k > 0 and sc.pdtr(k - 1, mu) >= qi:
                k -= 1
        else:
            while sc.pdtr(k, mu) < qi:
                k += 1
        out[i] = k
    return out
