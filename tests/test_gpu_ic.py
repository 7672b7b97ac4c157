"""Iman-Conover on the GPU vs the reference (correlation.py:368-425).

Gate: the step-4 permutation indices and the output Y are bit-exact; the van der Waerden
scores S within 1e-14 relative (device ndtri vs scipy's), correlated scores CS and the rank
correlation E within 1e-11 (different but exact-rounding reductions).  Golden cases come
from the reference run (tests/golden/ic.npz); larger N is checked against oracle.ic.
"""

import numpy as np
import pytest
import scipy.stats

from conftest import assert_close, golden

pytestmark = pytest.mark.gpu

CASES = ["cfg2", "cfg3", "ties"]


@pytest.fixture(scope="module")
def icz():
    return golden("ic.npz")


@pytest.mark.parametrize("tag", CASES)
def test_ic_golden_intermediates(gpu, icz, tag):
    from probabilit_amd.correlation import ImanConover

    X, C = icz[f"{tag}_X"], icz[f"{tag}_C"]
    Y, S, CS, idx, E = ImanConover().set_target(C)._call_debug(X)
    assert_close(S, icz[f"{tag}_S"], rtol=1e-14, atol=1e-300, what="scores")
    if f"{tag}_E" in icz:
        assert_close(E, icz[f"{tag}_E"], rtol=1e-11, atol=1e-13, what="corrcoef")
    assert_close(CS, icz[f"{tag}_CS"], rtol=1e-11, atol=1e-12, what="correlated scores")
    np.testing.assert_array_equal(idx, icz[f"{tag}_idx"])
    np.testing.assert_array_equal(Y, icz[f"{tag}_Y"])


@pytest.mark.parametrize("tag", ["toy", "normal", "lognormal", "readme", "cfg2", "cfg3", "ties"])
def test_ic_golden_outputs(gpu, icz, tag):
    from probabilit_amd.correlation import ImanConover

    C = icz["toy_C"] if tag in ("toy", "normal", "lognormal") else icz[f"{tag}_C"]
    Y = ImanConover().set_target(C)(icz[f"{tag}_X"])
    np.testing.assert_array_equal(Y, icz[f"{tag}_Y"])


def test_ic_doctest_statistics(gpu, icz):
    """correlation.py:335-361 and README.md:121-130 quote these correlations."""
    from probabilit_amd.correlation import ImanConover

    t = ImanConover().set_target(icz["toy_C"])
    assert round(scipy.stats.pearsonr(*t(icz["toy_X"]).T).statistic, 6) == 0.816497
    assert round(scipy.stats.pearsonr(*t(icz["normal_X"]).T).statistic, 6) == 0.697701
    assert round(scipy.stats.pearsonr(*t(icz["lognormal_X"]).T).statistic, 6) == 0.592541
    r = ImanConover().set_target(icz["readme_C"])(icz["readme_X"])
    assert format(scipy.stats.pearsonr(*r.T).statistic, ".8f") == "0.27965287"


@pytest.mark.parametrize("n,k", [(50_000, 3), (262_144, 32), (1_000_003, 8)])
def test_ic_vs_oracle_bit_exact_indices(gpu, n, k):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    X = ppf_columns(lhs_quantiles(n, k, 7), cfg_dists(k))
    C = cfg3_corr(k)
    ref = oic.iman_conover(X, C)
    Y, S, CS, idx, E = ImanConover().set_target(C)._call_debug(X)
    mism = int((idx != ref["idx"]).sum())
    assert mism == 0, f"{mism} step-4 index mismatches"
    np.testing.assert_array_equal(Y, ref["Y"])
    assert_close(S, ref["S"], rtol=1e-14, atol=1e-300, what="scores")


@pytest.mark.parametrize("n,k", [(8_192, 2), (3_000_017, 4)])
def test_ic_outputs_vs_oracle_placement_path(gpu, n, k):
    """Y without the debug outputs (the production step 4: 32-bit code sort, run fix-up and
    the LDS row placement with 0 / 2 bucket passes) equals the oracle's Y exactly."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    X = ppf_columns(lhs_quantiles(n, k, 5), cfg_dists(k))
    C = cfg3_corr(k)
    ref = oic.iman_conover(X, C)
    Y = ImanConover().set_target(C)(X)
    np.testing.assert_array_equal(Y, ref["Y"])


def test_ic_exact_ties_in_correlated_scores(gpu):
    """Duplicated rows of X give identical scores rows, so CS has exact ties: their 'average'
    rank is shared (correlation.py:422), which the placement path must reproduce."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(4)
    X = rng.normal(size=(20_000, 3))
    X[100:140] = X[0:40]  # 40 duplicated rows -> 40 tie runs of length 2 in every CS column
    X[7000:7003] = X[9000]  # and a run of 4
    C = cfg3_corr(3)
    ref = oic.iman_conover(X, C)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), ref["Y"])


def test_ic_properties_large(gpu):
    """N = 4M, K = 32: marginals preserved exactly, rank correlation near the target."""
    import torch

    from oracle.pipeline import cfg3_corr
    from probabilit_amd import native
    from probabilit_amd.correlation import ImanConover

    n, k = 4_000_000, 32
    C = cfg3_corr(k)
    X = native.fill_lhs(11, n, k, return_device=True).T.contiguous()  # (n, k) uniforms on device
    Y = ImanConover().set_target(C)(X)
    Xs, Ys = torch.sort(X, dim=0).values, torch.sort(Y, dim=0).values
    assert torch.equal(Xs, Ys)
    sub = Y[:: 40].cpu().numpy()
    rho = scipy.stats.spearmanr(sub).statistic
    assert np.abs(rho - C).max() < 0.02


def test_ic_reference_error_cases(gpu):
    from probabilit_amd.correlation import CorrelatorError, ImanConover

    with pytest.raises(ValueError):  # unity correlation in ranks (test_iman_conover.py:200-210)
        ImanConover().set_target(np.identity(2))(np.array([[1.0, 1], [2.0, 1.1], [2.1, 3]]))
    with pytest.raises(ValueError):
        ImanConover().set_target(np.identity(2))(np.array([[1.0, np.nan], [2.0, 1.1], [2.1, 3], [4, 5]]))
    with pytest.raises(CorrelatorError):
        ImanConover()(np.ones((5, 2)))
    with pytest.raises(ValueError):
        ImanConover().set_target(np.identity(3))(np.random.default_rng(0).normal(size=(10, 2)))


def test_ic_identity_target_keeps_decorrelated_data(gpu):
    """test_iman_conover.py:178-198."""
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(42)
    X = rng.normal(size=(5, 3))
    mean = X.mean(0)
    L = np.linalg.cholesky(np.cov(X, rowvar=False))
    import scipy.linalg

    X = mean + scipy.linalg.solve_triangular(L, (X - mean).T, lower=True).T
    Y = ImanConover().set_target(np.identity(3))(X)
    assert np.allclose(X, Y)


@pytest.mark.parametrize("seed", range(10))
def test_ic_marginals_and_distance(gpu, seed):
    """test_iman_conover.py:145-176, 10 of its 100 seeds (K up to 99)."""
    import scipy.linalg

    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(seed)
    k = int(rng.integers(2, 100))
    n = k * 10
    A = rng.normal(size=(k * 2, k))
    C = 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(k)
    X = rng.normal(size=(n, k))
    Y = ImanConover().set_target(C)(X)
    for j in range(k):
        assert np.allclose(np.sort(X[:, j]), np.sort(Y[:, j]))
    before = scipy.linalg.norm(np.corrcoef(X, rowvar=False) - C, ord="fro")
    after = scipy.linalg.norm(np.corrcoef(Y, rowvar=False) - C, ord="fro")
    assert after <= before


@pytest.mark.parametrize("n", [1, 2, 17, 4096, 4097, 100_000])
def test_rankdata_average_with_ties(gpu, n):
    from probabilit_amd.correlation import rankdata

    rng = np.random.default_rng(n)
    for x in (rng.integers(0, max(2, n // 10), n).astype(float), rng.normal(size=n), np.zeros(n),
              np.r_[np.full(n // 2, -0.0), np.zeros(n - n // 2)]):
        np.testing.assert_array_equal(rankdata(x), scipy.stats.rankdata(x))
