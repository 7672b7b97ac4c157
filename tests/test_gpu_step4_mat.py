"""Step 4 of MATERIALISED columns (X given: the operator API, the reference LHS stream) through the
generated columns' passes -- top-16 histogram, MSD code passes, bucket finish, row placement --
with sort(X)[p] gathered from the sorted column (k_place_sorted) instead of regenerated.
PBH_STEP4_MAT=msd selects that path (measured slower than the general path's per-column code sort
and value-carrying row placement, which stays the default); both must give the oracle's Y and
indices bit for bit."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def msd(monkeypatch):
    monkeypatch.setenv("PBH_STEP4_MAT", "msd")


@pytest.mark.parametrize("n,k,seed", [(50_000, 3, 7), (100_003, 8, 1), (300_017, 4, 5)])
def test_mat_msd_indices_bit_exact(gpu, msd, n, k, seed):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    X = ppf_columns(lhs_quantiles(n, k, seed), cfg_dists(k))
    C = cfg3_corr(k)
    ref = oic.iman_conover(X, C)
    Y, S, CS, idx, E = ImanConover().set_target(C)._call_debug(X)
    assert int((idx != ref["idx"]).sum()) == 0
    np.testing.assert_array_equal(Y, ref["Y"])


def test_mat_msd_exact_ties(gpu, msd):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(4)
    X = rng.normal(size=(20_000, 3))
    X[100:140] = X[0:40]
    X[7000:7003] = X[9000]
    C = cfg3_corr(3)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_mat_msd_discrete_columns(gpu, msd):
    """Integer-valued columns (long runs of equal X, so equal van der Waerden scores and exact CS
    ties the finish resolves to 'average' positions) and a spike that needs the adaptive code map."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(11)
    n = 40_000
    X = np.column_stack([rng.poisson(3.0, n).astype(float), rng.normal(size=n), rng.binomial(1, 0.3, n).astype(float),
                         rng.gamma(2.0, size=n)])
    C = cfg3_corr(4)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_mat_msd_long_runs_fall_back(gpu, msd):
    """40 identical rows: a run of equal codes beyond the finish, redone by the general path."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(9)
    X = rng.normal(size=(30_000, 2))
    X[5000:5040] = X[123]
    C = cfg3_corr(2)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_mat_msd_matches_general_large(gpu, monkeypatch):
    """n = 3M: identical Y from the MSD path and the general path, and the oracle's on the whole
    design."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    n, k = 3_000_000, 6
    X = ppf_columns(lhs_quantiles(n, k, 3), cfg_dists(k))
    C = cfg3_corr(k)
    monkeypatch.setenv("PBH_STEP4_MAT", "general")
    Y_g = ImanConover().set_target(C)(X)
    monkeypatch.setenv("PBH_STEP4_MAT", "msd")
    Y_m = ImanConover().set_target(C)(X)
    np.testing.assert_array_equal(Y_m, Y_g)
    np.testing.assert_array_equal(Y_m, oic.iman_conover(X, C)["Y"])
