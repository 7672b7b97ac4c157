"""PermutationCorrelator / CorrelationMatrix on the GPU (correlation.py:428-703, 757-921).

Parity, two ways:
* from the reference's own fixtures (tests/golden/permcorr.npz): output X, printed progress and
  the rng state after the call.  The initial correlation matrix comes from the device Gram
  (summation order differs from numpy's BLAS matmul by ~1e-15 relative), so this is exact
  unless some accept decision is a near-tie at that level -- none is, on these fixtures;
* from an identical initial state (the oracle's numpy CorrelationMatrix) and the identical swap
  stream: the device loop's decisions, permuted data and progress equal the oracle's bit for
  bit, at sizes up to N = 10^6, K = 32 (size-independent: the loop is exact arithmetic replay).
"""

import contextlib
import io
import json

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _cases():
    z = golden("permcorr.npz")
    meta = json.loads(str(z["meta"]))
    return z, meta, [k for k in meta if k != "subiters"]


@pytest.mark.parametrize("name", _cases()[2])
def test_permutation_correlator_matches_reference(gpu, name):
    from probabilit_amd.correlation import PermutationCorrelator

    z, meta, _ = _cases()
    m = meta[name]
    pc = PermutationCorrelator(**m["kwargs"])
    pc = pc.set_target(z[f"{name}_C"], weights=z[f"{name}_W"]) if m["weights"] else pc.set_target(z[f"{name}_C"])
    X = z[f"{name}_X"].copy()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        Y = pc(X)
    assert np.array_equal(X, z[f"{name}_X"]), "X was mutated"
    assert np.array_equal(Y, z[f"{name}_Y"]), f"{name}: {np.sum(Y != z[name + '_Y'])} entries differ"
    assert buf.getvalue() == m["stdout"]
    ref = json.loads(m["rng_after"])
    st = pc.rng.bit_generator.state
    assert str(st["state"]["state"]) == ref["state"] and st["has_uint32"] == ref["has_uint32"]
    assert st["uinteger"] == ref["uinteger"]


@pytest.mark.parametrize("n,k,iters,ctype,tol", [(500, 4, 60, "pearson", 1e-9), (20_000, 16, 40, "spearman", 1e-9),
                                                 (1_000_000, 32, 30, "pearson", 1e-9), (3000, 8, 400, "pearson", 0.1),
                                                 (4000, 100, 12, "pearson", 1e-9)])
def test_device_climb_equals_oracle_from_same_state(gpu, n, k, iters, ctype, tol):
    import torch

    from oracle.permcorr import ReferenceSwaps, climb, initial_state
    from probabilit_amd import device
    from probabilit_amd.correlation import PermutationCorrelator, SwapIndexGenerator

    g = np.random.default_rng(n + k)
    X = g.gamma(2.0, size=(n, k)) + g.normal(size=(n, 1))
    if ctype == "spearman":
        X[:, 0] = g.poisson(2.0, size=n)
    A = g.normal(size=(3 * k, k))
    C = 0.6 * np.corrcoef(A, rowvar=False) + 0.4 * np.eye(k)
    Xo, Xs, _, den, corr = initial_state(X, ctype)
    xo_d = device.to_device(np.ascontiguousarray(Xo.T))
    xs_d = xo_d if ctype == "pearson" else device.to_device(np.ascontiguousarray(Xs.T))
    pc = PermutationCorrelator(iterations=iters, tol=tol, seed=3, verbose=True).set_target(C)
    corr0 = corr.copy()
    gen = SwapIndexGenerator(pc.rng, n)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        pc._climb(xs_d, None if ctype == "pearson" else xo_d, corr0, den, gen)
    rng = np.random.default_rng(3)
    swaps = ReferenceSwaps(rng, n, iters)
    Wn = np.ones_like(C) / C.size
    Yref, lines, steps = climb(Xo, Xs, corr, den, C, Wn, iters, tol, swaps, verbose_every=iters // 10)
    torch.cuda.synchronize()
    assert np.array_equal(device.to_host(xo_d).T, Yref)
    assert buf.getvalue() == "".join(s + "\n" for s in lines)
    assert pc.rng.bit_generator.state == rng.bit_generator.state
    if tol > 1e-6:
        assert steps < iters * k, "expected an early stop"


def test_correlation_matrix_docstring_and_commit(gpu):
    """correlation.py:779-817 plus a spearman commit, against the reference's values."""
    from probabilit_amd.correlation import CorrelationMatrix

    z = golden("permcorr.npz")
    cm = CorrelationMatrix(z["cm_X"])
    np.testing.assert_allclose(cm[:, :], z["cm_corr0"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(cm.update_column(col=0, i=2, j=3), z["cm_update_0_2_3"], rtol=0, atol=1e-14)
    np.testing.assert_allclose(cm.update_column(col=0, i=[0, 1], j=[2, 3]), z["cm_update_0_01_23"], rtol=0,
                               atol=1e-14)
    cm.commit(col=1, i=[4, 5], j=[6, 8])
    np.testing.assert_allclose(cm[:, :], z["cm_after_commit"], rtol=0, atol=1e-14)
    assert np.array_equal(cm.X, z["cm_X_after_commit"])
    with pytest.raises(ValueError, match="disjoint"):
        cm.update_column(col=0, i=[1, 2], j=[2, 3])
    cms = CorrelationMatrix(z["cms_X"], correlation_type="spearman")
    np.testing.assert_allclose(cms[:, :], z["cms_corr0"], rtol=0, atol=1e-14)
    cms.commit(col=2, i=[0, 7], j=[3, 29])
    np.testing.assert_allclose(cms[:, :], z["cms_after_commit"], rtol=0, atol=1e-14)
    assert np.array_equal(cms.X, z["cms_X_after_commit"])
    with pytest.raises(ValueError, match="constant"):
        CorrelationMatrix(np.ones((5, 2)))


def test_permutation_correlator_errors_and_device_tensors(gpu):
    import torch

    from probabilit_amd import device
    from probabilit_amd.correlation import CorrelatorError, PermutationCorrelator

    C = np.array([[1.0, 0.6], [0.6, 1.0]])
    X = np.random.default_rng(0).normal(size=(50, 2))
    with pytest.raises(CorrelatorError):
        PermutationCorrelator()(X)
    with pytest.raises(ZeroDivisionError):
        PermutationCorrelator(iterations=5).set_target(C)(X)
    with pytest.raises(ValueError):
        PermutationCorrelator().set_target(C)(np.ones((20, 2)))
    Xd = device.to_device(X)
    Yd = PermutationCorrelator(seed=1).set_target(C)(Xd)
    assert isinstance(Yd, torch.Tensor) and Yd.is_cuda
    assert np.array_equal(device.to_host(Xd), X), "device input was mutated"
    Yh = PermutationCorrelator(seed=1).set_target(C)(X)
    assert np.array_equal(device.to_host(Yd), Yh)
    for c in range(2):  # marginals preserved
        assert np.array_equal(np.sort(Yh[:, c]), np.sort(X[:, c]))


def test_dag_with_permutation_correlator(gpu):
    """correlator=<a PermutationCorrelator class> in Node.sample (modeling.py:505-507, 577-581):
    the DAG hands the correlator the uncorrelated samples; same result as calling it directly."""
    from probabilit_amd.correlation import PermutationCorrelator
    from probabilit_amd.modeling import Distribution, NoOp

    class Seeded(PermutationCorrelator):
        def __init__(self):
            super().__init__(iterations=300, seed=5)

    C = np.array([[1.0, 0.8], [0.8, 1.0]])
    a, b = Distribution("norm"), Distribution("expon")
    NoOp(a, b).correlate(a, b, corr_mat=C).sample(2000, random_state=0, method="lhs", correlator=Seeded)
    a2, b2 = Distribution("norm"), Distribution("expon")
    NoOp(a2, b2).sample(2000, random_state=0, method="lhs")
    X = np.column_stack([a2.samples_, b2.samples_])
    Y = Seeded().set_target(C)(X)
    assert np.array_equal(np.column_stack([a.samples_, b.samples_]), Y)
    assert np.corrcoef(Y, rowvar=False)[0, 1] > np.corrcoef(X, rowvar=False)[0, 1] + 0.2
