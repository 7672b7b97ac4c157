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


def _permcorr_cases():
    z = golden("permcorr.npz")
    meta = json.loads(str(z["meta"]))
    return z, meta, [k for k in meta if k != "subiters"]


def test_oracle_permutation_correlator_vs_reference():
    """oracle/permcorr.py restates PermutationCorrelator (correlation.py:473-703): the reference's
    output, printed progress and rng state after the call, bit for bit, on every fixture."""
    from oracle.permcorr import permutation_correlate

    z, meta, cases = _permcorr_cases()
    for name in cases:
        m = meta[name]
        W = z[f"{name}_W"] if m["weights"] else None
        Y, text, rng = permutation_correlate(z[f"{name}_X"], z[f"{name}_C"], weights=W, **m["kwargs"])
        assert np.array_equal(Y, z[f"{name}_Y"]), name
        assert text == m["stdout"], name
        ref = json.loads(m["rng_after"])
        st = rng.bit_generator.state
        assert str(st["state"]["state"]) == ref["state"] and st["has_uint32"] == ref["has_uint32"], name


def test_swap_index_generator_host_stream():
    """The product's SwapIndexGenerator (host logic, no GPU) draws the reference's stream: the
    golden sizes sequence through a permutation exhaustion, and random size sequences against
    the oracle's call-per-step restatement, including the rng state afterwards."""
    from oracle.permcorr import SwapStream, subiters
    from probabilit_amd.correlation import PermutationCorrelator, SwapIndexGenerator

    z, meta, _ = _permcorr_cases()
    sg = SwapIndexGenerator(np.random.default_rng(11), 9)
    flat = np.concatenate([np.concatenate(sg(int(s))) for s in z["swapgen_n9_sizes"]])
    assert np.array_equal(flat, z["swapgen_n9_flat"])
    for n, ref in meta["subiters"].items():
        assert [PermutationCorrelator.subiters(int(n), i) for i in range(1, int(n) + 1)] == ref
        assert [subiters(int(n), i) for i in range(1, int(n) + 1)] == ref
    g = np.random.default_rng(5)
    for n in (2, 3, 7, 10, 64, 1000):
        sizes = g.integers(1, 12, size=300)
        a, b = np.random.default_rng(n), np.random.default_rng(n)
        gen, ref = SwapIndexGenerator(a, n), SwapStream(b, n)
        flat, offs = gen._take_many(sizes)
        want = [np.concatenate(ref(int(s))) for s in sizes]
        assert np.array_equal(np.diff(offs), [len(w) for w in want])
        assert np.array_equal(flat, np.concatenate(want))
        assert a.bit_generator.state == b.bit_generator.state
        assert np.array_equal(gen.permutation, ref.perm)


def test_permutation_correlator_validation():
    """Constructor checks of correlation.py:561-575 (including the tol check's precedence)."""
    from probabilit_amd.correlation import PermutationCorrelator

    with pytest.raises(ValueError):
        PermutationCorrelator(weights=np.array([[1.0, 0.0]]))
    with pytest.raises(ValueError):
        PermutationCorrelator(iterations=-1)
    with pytest.raises(ValueError):
        PermutationCorrelator(iterations=2.0)
    with pytest.raises(ValueError):
        PermutationCorrelator(tol=1)
    PermutationCorrelator(tol=-1)  # sic: an int tol <= 0 passes the reference's check
    with pytest.raises(TypeError):
        PermutationCorrelator(seed=1.5)
    with pytest.raises(TypeError):
        PermutationCorrelator(verbose=1)
    pc = PermutationCorrelator().set_target(np.array([[1.0, 0.5], [0.5, 1.0]]), weights=np.array([[1, 2], [2, 1]]))
    assert np.allclose(pc.weights, np.array([[1, 2], [2, 1]]) / 6)
    assert pc._error(np.eye(2), pc.C) == pytest.approx(np.sqrt(2 / 6 * 0.25))


def test_threaded_oracle_is_bit_identical():
    """The thread-pooled forms used by the large parity tests (oracle.ic threads=,
    oracle.pipeline.ppf_columns threads=) give exactly the sequential results."""
    from oracle import ic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns

    n, d = 30_000, 16
    Q = lhs_quantiles(n, d, 5)
    X1 = ppf_columns(Q, cfg_dists(d))
    X4 = ppf_columns(Q, cfg_dists(d), threads=4, chunk=7_001)
    np.testing.assert_array_equal(X1, X4)
    a, b = ic.iman_conover(X1, cfg3_corr(d)), ic.iman_conover(X1, cfg3_corr(d), threads=4)
    for key in ("Y", "S", "E", "CS", "idx"):
        np.testing.assert_array_equal(a[key], b[key], err_msg=key)
