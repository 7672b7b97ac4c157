"""Step 4's code sort through the top-16-bit buckets (k_code_buckets: two one-sweep passes +
a per-bucket LDS finish that also orders equal-code runs) against the oracle and against the
four-pass path.  PBH_STEP4=buckets forces the bucket path below its default size range
(n >= 2^22), PBH_STEP4=lsd forces the four-pass path."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture
def buckets(monkeypatch):
    monkeypatch.setenv("PBH_STEP4", "buckets")


@pytest.mark.parametrize("n,k", [(50_000, 3), (262_144, 32), (100_003, 8)])
def test_bucket_path_indices_bit_exact(gpu, buckets, n, k):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    X = ppf_columns(lhs_quantiles(n, k, 7), cfg_dists(k))
    C = cfg3_corr(k)
    ref = oic.iman_conover(X, C)
    Y, S, CS, idx, E = ImanConover().set_target(C)._call_debug(X)
    assert int((idx != ref["idx"]).sum()) == 0
    np.testing.assert_array_equal(Y, ref["Y"])


@pytest.mark.parametrize("n,k", [(8_192, 2), (300_017, 4)])
def test_bucket_path_placement_vs_oracle(gpu, buckets, n, k):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    X = ppf_columns(lhs_quantiles(n, k, 5), cfg_dists(k))
    C = cfg3_corr(k)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_bucket_path_exact_ties(gpu, buckets):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(4)
    X = rng.normal(size=(20_000, 3))
    X[100:140] = X[0:40]
    X[7000:7003] = X[9000]
    C = cfg3_corr(3)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_bucket_path_long_runs_fall_back(gpu, buckets):
    """A run of > 16 equal codes (here 40 identical rows) takes the 64-bit fallback."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    rng = np.random.default_rng(9)
    X = rng.normal(size=(30_000, 2))
    X[5000:5040] = X[123]
    C = cfg3_corr(2)
    np.testing.assert_array_equal(ImanConover().set_target(C)(X), oic.iman_conover(X, C)["Y"])


def test_bucket_and_four_pass_paths_agree_large(gpu, monkeypatch):
    """n = 5M (the bucket path's default range): identical Y from both paths, and the oracle's
    indices on a 4-column slice."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.correlation import ImanConover

    n, k = 5_000_000, 4
    X = ppf_columns(lhs_quantiles(n, k, 3), cfg_dists(k))
    C = cfg3_corr(k)
    monkeypatch.setenv("PBH_STEP4", "lsd")
    Y_lsd = ImanConover().set_target(C)(X)
    monkeypatch.delenv("PBH_STEP4")
    Y_b = ImanConover().set_target(C)(X)
    np.testing.assert_array_equal(Y_b, Y_lsd)
    np.testing.assert_array_equal(Y_b, oic.iman_conover(X, C)["Y"])
