"""Statistical checks of the native LHS stream, the quantile source of every headline number
(`method="lhs"`, modeling.py:480,488 -> pbh_rng.h: stratum pi(row) from a 4-round keyed FE2
Feistel bijection whose round keys come from Philox4x32-10, jitter of stratum t from SplitMix64
output t keyed by (seed, column)).

The reference's scipy LatinHypercube draws d independent uniform permutations and independent
jitters.  A keyed bijection is not a uniform random permutation, so these tests bound what a user
of uncorrelated columns (BASELINE config 2: no correlation step to wash structure out) would see,
at N = 1e7 for several seeds and for adjacent seeds:

* pairwise Pearson correlation of the strata (= Spearman of the samples) and of the cfg2 samples
  between every column pair: |r| < 5 / sqrt(N);
* no correlation between the row index and the stratum, nor between the strata of adjacent rows
  (serial structure of pi), per column: |r| < 5 / sqrt(N);
* chi-square of the 64 x 64 stratum-cell occupancy for every column pair, for adjacent rows of
  one column, and for the same column under adjacent seeds: two-sided p > 1e-6 (a lattice would
  show up as too small a statistic, clustering as too large);
* the jitter's uniformity inside the strata (1 024-bin chi-square).

DESIGN.md §4 justifies the Feistel round count with these results.
"""

import numpy as np
import pytest
import scipy.stats

pytestmark = pytest.mark.gpu

N = 10_000_000
D = 8
SEEDS = [0, 1, 2, 12345]
BOUND = 5.0 / np.sqrt(N)
CELLS = 64
P_MIN = 1e-6


def _quantiles(seed, d=D):
    from probabilit_amd import native

    return native.fill_lhs(seed, N, d, return_device=True)  # (d, N) on the device


def _strata(q):
    import torch

    return torch.clamp(torch.floor(q * N), max=N - 1)


def _corr(a, b):
    import torch

    a = a - a.mean()
    b = b - b.mean()
    return float((a * b).sum() / torch.sqrt((a * a).sum() * (b * b).sum()))


def _chi2_cells(sa, sb):
    """Two-sided p of the 64 x 64 occupancy of the stratum pairs (sa, sb) (the margins of an LHS
    column are exact, so the statistic has (64 - 1)^2 degrees of freedom)."""
    import torch

    ia = (sa * CELLS / N).long().clamp(max=CELLS - 1)
    ib = (sb * CELLS / N).long().clamp(max=CELLS - 1)
    counts = torch.bincount(ia * CELLS + ib, minlength=CELLS * CELLS).double()
    expected = float(sa.numel()) / (CELLS * CELLS)
    stat = float(((counts - expected) ** 2).sum() / expected)
    dof = (CELLS - 1) ** 2
    return min(scipy.stats.chi2.sf(stat, dof), scipy.stats.chi2.cdf(stat, dof)), stat


@pytest.mark.parametrize("seed", SEEDS)
def test_strata_pairwise_uncorrelated_and_cells_uniform(gpu, seed):
    s = _strata(_quantiles(seed))
    worst_r, worst_p = 0.0, 1.0
    for i in range(D):
        for j in range(i + 1, D):
            r = _corr(s[i], s[j])
            p, stat = _chi2_cells(s[i], s[j])
            worst_r, worst_p = max(worst_r, abs(r)), min(worst_p, p)
            assert abs(r) < BOUND, (seed, i, j, r)
            assert p > P_MIN, (seed, i, j, stat)
    print(f"seed {seed}: max |rank corr| {worst_r:.2e} (bound {BOUND:.2e}), min chi2 p {worst_p:.3g}")


@pytest.mark.parametrize("seed", SEEDS)
def test_no_row_or_serial_structure(gpu, seed):
    import torch

    s = _strata(_quantiles(seed))
    rows = torch.arange(N, dtype=torch.float64, device=s.device)
    for c in range(D):
        assert abs(_corr(rows, s[c])) < BOUND, (seed, c, "row index")
        assert abs(_corr(s[c][:-1], s[c][1:])) < BOUND, (seed, c, "lag 1")
        assert abs(_corr(s[c][:-2], s[c][2:])) < BOUND, (seed, c, "lag 2")
        p, stat = _chi2_cells(s[c][:-1], s[c][1:])
        assert p > P_MIN, (seed, c, "adjacent rows", stat)


@pytest.mark.parametrize("seed", SEEDS[:3])
def test_adjacent_seeds_independent(gpu, seed):
    a = _strata(_quantiles(seed))
    b = _strata(_quantiles(seed + 1))
    for c in range(D):
        assert abs(_corr(a[c], b[c])) < BOUND, (seed, c)
        p, stat = _chi2_cells(a[c], b[c])
        assert p > P_MIN, (seed, c, stat)
    # and across columns of the two seeds
    assert abs(_corr(a[0], b[1])) < BOUND


@pytest.mark.parametrize("seed", SEEDS[:2])
def test_jitter_uniform_within_strata(gpu, seed):
    import torch

    q = _quantiles(seed, 2)
    u = (_strata(q) + 1.0) - q * N  # scipy's (perm - u) / n: u in (0, 1]
    for c in range(2):
        bins = torch.bincount((u[c] * 1024).long().clamp(0, 1023), minlength=1024).double()
        e = N / 1024.0
        stat = float(((bins - e) ** 2).sum() / e)
        p = min(scipy.stats.chi2.sf(stat, 1023), scipy.stats.chi2.cdf(stat, 1023))
        assert p > P_MIN, (seed, c, stat)
        # jitter independent of the stratum and of the row
        assert abs(_corr(u[c], _strata(q)[c])) < BOUND


@pytest.mark.parametrize("seed", SEEDS[:2])
def test_cfg2_samples_uncorrelated(gpu, seed):
    """BASELINE config 2's eight uncorrelated leaves through Node.sample_device: Pearson of the
    samples between every pair below 5 / sqrt(N)."""
    from oracle.pipeline import cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
    NoOp(*ds).sample_device(N, random_state=seed, method="lhs")
    cols = [x.samples_device for x in ds]
    for i in range(8):
        for j in range(i + 1, 8):
            r = _corr(cols[i], cols[j])
            assert abs(r) < BOUND, (seed, i, j, r)
