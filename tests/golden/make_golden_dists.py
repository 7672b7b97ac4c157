"""Golden fixtures for the distributions beyond the base set (beta / PERT, truncnorm, binom,
bernoulli, the distributions.py constructors), produced by the REAL reference (stub-imported
as in make_golden.py; build container only).  Writes tests/golden/dists.npz.

    python tests/golden/make_golden_dists.py
"""

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import modeling  # noqa: E402  (reference, stub-imported)
import probabilit.distributions as dists  # noqa: E402


def main():
    out = {}
    D = modeling.Distribution
    out["pert"] = dists.PERT(0, 6, 10).sample(2000, random_state=0)
    out["tnorm"] = dists.TruncatedNormal(loc=0, scale=1, low=3, high=3.3).sample(2000, random_state=0)
    out["tnorm_mid"] = dists.TruncatedNormal(loc=1, scale=2, low=-2, high=5).sample(2000, random_state=1,
                                                                                     method="lhs")
    out["lognorm_ms"] = dists.Lognormal(mean=2, std=1).sample(999, random_state=0)
    out["lognorm_comp"] = dists.Lognormal(mean=D("expon", scale=1), std=1).sample(500, random_state=0)
    out["tri"] = dists.Triangular(low=1, mode=5, high=9).sample(1000, random_state=3)
    out["binom"] = D("binom", n=20, p=0.3).sample(3000, random_state=2)
    out["bern"] = D("bernoulli", p=0.25).sample(3000, random_state=2)
    out["beta_small"] = D("beta", 0.5, 0.5).sample(2000, random_state=5)
    out["composite"] = D("beta", a=D("uniform", loc=1, scale=3), b=2.0).sample(1500, random_state=7)
    np.savez_compressed(os.path.join(HERE, "dists.npz"), **out)
    print({k: (v.shape, v.dtype) for k, v in out.items()})


if __name__ == "__main__":
    main()
