"""Pin the oracle (test infrastructure) to the reference's golden vectors (CPU only)."""

import json

import numpy as np
import pytest
import scipy
import scipy.stats

from conftest import golden


def test_fixture_environment_matches():
    meta = json.loads(str(golden("dag.npz")["meta"]))
    assert meta["scipy"] == scipy.__version__, "fixtures were made with another scipy"
    assert meta["numpy"] == np.__version__


def test_pcg64_lhs_restatement_bit_exact():
    from oracle.streams import lhs_reference

    z = golden("streams.npz")
    s = [int(x) for x in z["lhs_d8_s0_state"]]
    state, inc = (s[0] << 64) | s[1], (s[2] << 64) | s[3]
    q = lhs_reference((state, inc), 4096, 8)
    np.testing.assert_array_equal(q, z["lhs_d8_s0_n4096"])


def test_lhs_restatement_matches_scipy_engine():
    from oracle.streams import PCG64, lhs_reference

    eng = scipy.stats.qmc.LatinHypercube(d=3, rng=123)
    g = PCG64.from_numpy(eng.rng)
    np.testing.assert_array_equal(lhs_reference((g.state, g.inc), 1000, 3), golden("streams.npz")["lhs_d3_s123_n1000"])


@pytest.mark.parametrize("d,seed,n", [(20, 0, 4096), (5, 7, 1000), (32, 1, 512)])
def test_sobol_closed_form_bit_exact(d, seed, n):
    from oracle.streams import sobol_closed_form

    z = golden("streams.npz")
    q = sobol_closed_form(z[f"sobol_d{d}_s{seed}_sv"], z[f"sobol_d{d}_s{seed}_shift"], n)
    np.testing.assert_array_equal(q, z[f"sobol_d{d}_s{seed}_n{n}"])


def test_oracle_ppf_matches_golden():
    from oracle.ppf import ppf

    z = golden("ppf.npz")
    for name, (dist, kw) in json.loads(str(z["meta"])).items():
        np.testing.assert_array_equal(ppf(dist, z["q"], **kw), z[name])


@pytest.mark.parametrize("mu", [0.5, 4.0, 30.0, 1000.0])
def test_poisson_smallest_k_definition(mu):
    """The device kernel's definition equals scipy's ceil(pdtrik) + correction."""
    from oracle.ppf import poisson_smallest_k

    q = scipy.stats.qmc.LatinHypercube(d=1, rng=int(mu)).random(2000)[:, 0]
    np.testing.assert_array_equal(poisson_smallest_k(q, mu), scipy.stats.poisson(mu).ppf(q))


@pytest.mark.parametrize("tag", ["cfg2", "cfg3", "ties"])
def test_oracle_iman_conover_intermediates(tag):
    from oracle.ic import iman_conover

    z = golden("ic.npz")
    r = iman_conover(z[f"{tag}_X"], z[f"{tag}_C"])
    np.testing.assert_array_equal(r["Y"], z[f"{tag}_Y"])
    np.testing.assert_array_equal(r["idx"], z[f"{tag}_idx"])
    np.testing.assert_array_equal(r["S"], z[f"{tag}_S"])
    np.testing.assert_array_equal(r["CS"], z[f"{tag}_CS"])


def test_oracle_ties_quirk_not_permutation():
    """discrete leading columns make the step-4 index a non-permutation."""
    z = golden("ic.npz")
    idx = z["ties_idx"]
    assert len(np.unique(idx[:, 0])) < idx.shape[0]
    assert not np.array_equal(np.sort(z["ties_Y"][:, 1]), np.sort(z["ties_X"][:, 1]))


def test_oracle_rankdata_matches_scipy():
    from oracle.ic import rankdata_average

    rng = np.random.default_rng(0)
    for x in (rng.integers(0, 50, 5000).astype(float), rng.normal(size=5000), np.zeros(7)):
        np.testing.assert_array_equal(rankdata_average(x), scipy.stats.rankdata(x))


def test_oracle_pipelines_reproduce_fixtures():
    from oracle.pipeline import cfg3_corr, mutual_fund

    z = golden("dag.npz")
    np.testing.assert_array_equal(mutual_fund(z["fund_Q"]), z["fund_sink"])
    np.testing.assert_array_equal(mutual_fund(z["fund999_Q"]), z["fund999_sink"])
    np.testing.assert_array_equal(cfg3_corr(8), z["corr8_C"])


def test_oracle_correlators_vs_reference():
    """oracle/correlators.py restates Cholesky.__call__ / decorrelate on the same numpy calls:
    identical to the reference's outputs (tests/golden/correlators.npz)."""
    from oracle.correlators import cholesky_transform, decorrelate

    z = golden("correlators.npz")
    for tag in ("9x2", "500x3", "2000x8"):
        X, C = z[f"chol_X_{tag}"], z[f"chol_C_{tag}"]
        np.testing.assert_allclose(cholesky_transform(X, C), z[f"chol_Y_{tag}"], rtol=1e-14, atol=1e-14)
        np.testing.assert_allclose(decorrelate(X), z[f"decor_Y_{tag}"], rtol=1e-14, atol=1e-14)
        np.testing.assert_allclose(decorrelate(X, remove_variance=False), z[f"decor_keepvar_Y_{tag}"], rtol=1e-14,
                                   atol=1e-14)
