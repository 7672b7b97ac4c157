"""Drop-in for probabilit.distributions (src/probabilit/distributions.py @ 2025-09-19): the
convenience constructors, each returning a `Distribution` node whose inverse CDF runs on the
GPU (norm / uniform / triang / lognorm in pbh_ppf.hip, beta / truncnorm in pbh_ppf_ext.hip).

Only parameter conversion happens here (on the host, once per node): PERT -> beta shapes,
(mean, std) -> lognormal (s, scale) as DAG transforms, and the two-equation percentile fit of
Triangular.
"""

import warnings

import numpy as np

from .modeling import Distribution, Exp, Log, Sign

__all__ = ["Uniform", "Normal", "TruncatedNormal", "Lognormal", "PERT", "Triangular"]


def Uniform(min=0, max=1):
    """Uniform on [min, max) (distributions.py:7-9)."""
    return Distribution("uniform", loc=min, scale=max - min)


def Normal(loc, scale):
    """Normal with mean `loc` and standard deviation `scale` (distributions.py:12-14)."""
    return Distribution("norm", loc=loc, scale=scale)


def TruncatedNormal(loc, scale, low, high):
    """Normal(loc, scale) restricted to [low, high) (distributions.py:17-29): scipy's truncnorm
    takes the bounds in standard units."""
    return Distribution("truncnorm", a=(low - loc) / scale, b=(high - loc) / scale, loc=loc, scale=scale)


class Lognormal(Distribution):
    """Lognormal whose own mean and standard deviation are `mean` and `std` (numbers or nodes;
    distributions.py:32-75).  With v = sign(std) std^2 (a negative std fails downstream):
    sigma^2 = log(1 + v / mean^2), mu = log(mean) - sigma^2 / 2, then lognorm(s=sigma,
    scale=exp(mu)); the conversion is part of the DAG, so composite parameters work."""

    def __init__(self, mean, std):
        variance = Sign(std) * std**2
        sigma_squared = Log(1 + variance / (mean**2))
        super().__init__("lognorm", s=sigma_squared ** (1 / 2), scale=Exp(Log(mean) - sigma_squared / 2))

    @classmethod
    def from_log_params(cls, mu, sigma):
        """Lognormal from the mean `mu` and standard deviation `sigma` of log(X)."""
        return Distribution("lognorm", s=sigma, scale=Exp(mu))


def _pert_to_beta(minimum, mode, maximum, gamma=4.0):
    """(a, b, loc, scale) of the beta distribution behind PERT(minimum, mode, maximum, gamma)
    (distributions.py:187-215)."""
    if not (minimum < mode < maximum):
        raise ValueError(f"Must have {minimum=} < {mode=} < {maximum=}")
    if gamma <= 0:
        raise ValueError(f"Gamma must be positive, got {gamma=}")
    width = maximum - minimum
    return (1 + gamma * (mode - minimum) / width, 1 + gamma * (maximum - mode) / width, minimum, width)


def PERT(minimum, mode, maximum, gamma=4.0):
    """PERT distribution as the equivalent scaled beta (distributions.py:78-94)."""
    a, b, loc, scale = _pert_to_beta(minimum, mode, maximum, gamma=gamma)
    return Distribution("beta", a=a, b=b, loc=loc, scale=scale)


def _triangular_cdf(x, lo, hi, mode):
    if x <= lo:
        return x * 0
    if x >= hi:
        return x * 0 + 1.0
    if x <= mode:
        return (x - lo) ** 2 / ((hi - lo) * (mode - lo))
    return 1 - (hi - x) ** 2 / ((hi - lo) * (hi - mode))


def _fit_triangular_distribution(low, mode, high, low_perc=0.10, high_perc=0.90):
    """(loc, scale, c) of the triangular distribution with the given mode whose CDF is low_perc
    at `low` and high_perc at `high` (distributions.py:137-184): scipy.optimize.fsolve on the two
    support ends, started outside [low, high]."""
    import scipy.optimize

    def residual(ends):
        lo, hi = ends
        return (_triangular_cdf(low, lo, hi, mode) - low_perc, _triangular_cdf(high, lo, hi, mode) - high_perc)

    lo, hi = scipy.optimize.fsolve(residual, (low - abs(mode - low), high + abs(high - mode)))
    rmse = np.sqrt(np.sum(np.array(residual([lo, hi])) ** 2))
    if rmse > 1e-6:
        warnings.warn(f"Optimization of Triangular params has {rmse=}")
    return float(lo), float(hi - lo), float((mode - lo) / (hi - lo))


def Triangular(low, mode, high, low_perc=0.1, high_perc=0.9):
    """Triangular distribution with the given mode whose low_perc / high_perc percentiles are
    `low` / `high` (distributions.py:97-134).  Numbers only (no composite parameters)."""
    if not (low < mode < high):
        raise ValueError(f"Must have {low=} < {mode=} < {high=}")
    if not ((0 <= low_perc <= 1.0) and (0 <= high_perc <= 1.0)):
        raise ValueError("Percentiles must be between 0 and 1.")
    if np.isclose(low_perc, 0.0) and np.isclose(high_perc, 1.0):
        loc, scale, c = low, high - low, (mode - low) / (high - low)
    else:
        loc, scale, c = _fit_triangular_distribution(low, mode, high, low_perc=low_perc, high_perc=high_perc)
    return Distribution("triang", loc=loc, scale=scale, c=c)
