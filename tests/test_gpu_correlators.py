"""Cholesky correlator and decorrelate on the GPU (correlation.py:205-285, 706-754) against
the oracle restatement (oracle/correlators.py) and the reference's docstring pins.

Tolerance: the reference's covariance / products are BLAS dgemm calls whose summation order is
library dependent, so floating-point parity is 1e-10 relative (the north_star's ppf gate)."""

import numpy as np
import pytest

from conftest import assert_close

pytestmark = pytest.mark.gpu


def _corr(k, seed):
    A = np.random.default_rng(seed).normal(size=(3 * k, k))
    return 0.8 * np.corrcoef(A, rowvar=False) + 0.2 * np.eye(k)


@pytest.mark.parametrize("n,k", [(9, 2), (1000, 3), (20_000, 8), (4096, 32), (700, 40)])
def test_cholesky_matches_oracle(gpu, n, k):
    from oracle.correlators import cholesky_transform
    from probabilit_amd.correlation import Cholesky

    rng = np.random.default_rng(n + k)
    X = rng.gamma(2.0, size=(n, k)) + rng.normal(size=(n, 1))
    C = _corr(k, k)
    Y = Cholesky().set_target(C)(X)
    ref = cholesky_transform(X, C)
    assert_close(Y, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max(), what="Cholesky")


def test_cholesky_docstring_pins(gpu):
    """correlation.py:217-243."""
    import scipy.stats

    from probabilit_amd.correlation import Cholesky

    X = np.random.default_rng(4).normal(size=(9, 2))
    Xt = Cholesky().set_target(np.array([[1, 0.7], [0.7, 1]]))(X)
    assert round(float(scipy.stats.pearsonr(*Xt.T).statistic), 6) == 0.7
    np.testing.assert_allclose(np.mean(Xt, axis=0), [-0.63531692, 0.70114825], rtol=1e-7)
    np.testing.assert_allclose(np.std(Xt, axis=0), [1.11972638, 0.75668173], rtol=1e-7)


def test_cholesky_in_dag_docstring(gpu):
    """modeling.py:459-466: correlator=Cholesky through Node.sample."""
    import scipy.stats

    from probabilit_amd.correlation import Cholesky
    from probabilit_amd.modeling import Distribution

    a, b = Distribution("uniform"), Distribution("expon")
    result = (a + b).correlate(a, b, corr_mat=np.array([[1, 0.6], [0.6, 1]]))
    result.sample(25, random_state=0, correlator=Cholesky)
    assert abs(float(scipy.stats.pearsonr(a.samples_, b.samples_).statistic) - 0.6) < 1e-6
    assert f"{float(np.min(b.samples_)):.5f}" == "-0.35283"
    result.sample(25, random_state=0, correlator="cholesky")
    assert f"{float(np.min(b.samples_)):.5f}" == "-0.35283"


def test_cholesky_validation(gpu):
    from probabilit_amd.correlation import Cholesky, CorrelatorError

    with pytest.raises(CorrelatorError):
        Cholesky()(np.zeros((5, 2)))
    c = Cholesky().set_target(np.eye(2))
    with pytest.raises(ValueError):
        c(np.zeros((2, 2)))  # N <= K
    with pytest.raises(ValueError):
        c(np.zeros((5, 3)))  # K mismatch


@pytest.mark.parametrize("remove_variance", [True, False])
@pytest.mark.parametrize("n,k", [(3, 2), (500, 4), (10_000, 16)])
def test_decorrelate_matches_oracle(gpu, n, k, remove_variance):
    from oracle.correlators import decorrelate as ref_decorrelate
    from probabilit_amd.correlation import decorrelate

    if n == 3:
        X = np.array([[1.0, 1.0], [2.0, 1.1], [2.1, 3.0]])
    else:
        X = np.random.default_rng(k).normal(size=(n, k)) @ np.linalg.cholesky(_corr(k, 1)).T + 3.0
    Y = decorrelate(X, remove_variance=remove_variance)
    ref = ref_decorrelate(X, remove_variance=remove_variance)
    assert_close(Y, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max(), what="decorrelate")


def test_decorrelate_docstring(gpu):
    """correlation.py:709-743."""
    from probabilit_amd.correlation import decorrelate

    X = np.array([[1.0, 1.0], [2.0, 1.1], [2.1, 3.0]])
    D = decorrelate(X)
    np.testing.assert_array_equal(np.cov(D, rowvar=False).round(6), [[1.0, 0.0], [0.0, 1.0]])
    assert np.allclose(np.mean(X, axis=0), np.mean(D, axis=0))
    np.testing.assert_allclose(np.var(D, axis=0, ddof=1), [1.0, 1.0])
    D2 = decorrelate(X, remove_variance=False)
    np.testing.assert_array_equal(np.cov(D2, rowvar=False).round(6), [[0.246667, 0.0], [0.0, 0.846667]])


@pytest.mark.parametrize("tag", ["9x2", "500x3", "2000x8"])
def test_correlators_vs_reference_golden(gpu, tag):
    """Outputs the reference itself produced (tests/golden/correlators.npz)."""
    from conftest import golden
    from probabilit_amd.correlation import Cholesky, decorrelate

    z = golden("correlators.npz")
    X, C = z[f"chol_X_{tag}"], z[f"chol_C_{tag}"]
    for got, ref in [(Cholesky().set_target(C)(X), z[f"chol_Y_{tag}"]), (decorrelate(X), z[f"decor_Y_{tag}"]),
                     (decorrelate(X, remove_variance=False), z[f"decor_keepvar_Y_{tag}"])]:
        assert_close(got, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max(), what=tag)


def test_dag_streams_vs_reference_golden(gpu):
    """Node.sample with method=None (RandomState / Generator) and method='halton': the
    reference's own outputs at the same seeds (tests/golden/correlators.npz)."""
    from conftest import golden
    from probabilit_amd.modeling import Distribution

    z = golden("correlators.npz")
    a = Distribution("norm", loc=1.0, scale=2.0)
    b = Distribution("expon", scale=3.0)
    expr = a * b + 1.0
    assert_close(expr.sample(1000, random_state=0), z["dag_none_s0_n1000"], what="None/int")
    assert_close(expr.sample(513, random_state=4, method="halton"), z["dag_halton_s4_n513"], what="halton")
    assert_close(expr.sample(100, random_state=np.random.RandomState(3)), z["dag_none_rs_n100"], what="RandomState")
    assert_close(expr.sample(100, random_state=np.random.default_rng(3)), z["dag_none_gen_n100"], what="Generator")
