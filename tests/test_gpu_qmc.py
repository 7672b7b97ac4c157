"""Quantile generators on the GPU.

Sobol' is bit-exact with scipy.stats.qmc.Sobol (golden points from the reference run);
the native LHS is checked for the Latin-hypercube property exactly (one point per stratum
per column) and for shard independence (any row range regenerates bit-identically).
"""

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("d,seed,n", [(20, 0, 4096), (5, 7, 1000), (32, 1, 512)])
def test_sobol_bit_exact(gpu, d, seed, n):
    from probabilit_amd import native, qmc

    z = golden("streams.npz")
    sv, shift = qmc.sobol_setup(d, seed)
    q = native.fill_sobol(sv, shift, n)
    np.testing.assert_array_equal(q, z[f"sobol_d{d}_s{seed}_n{n}"])


def test_sobol_row_shards(gpu):
    from probabilit_amd import native, qmc

    sv, shift = qmc.sobol_setup(7, 3)
    full = native.fill_sobol(sv, shift, 10_000)
    part = native.fill_sobol(sv, shift, 3000, row0=5000)
    np.testing.assert_array_equal(part, full[5000:8000])


@pytest.mark.parametrize("n", [1, 2, 3, 1000, 65_537, 1_000_000])
def test_native_lhs_is_latin_hypercube(gpu, n):
    from probabilit_amd import native

    d = 4
    q = native.fill_lhs(99, n, d)
    assert q.shape == (n, d)
    assert np.all(q >= 0.0) and np.all(q < 1.0)
    for k in range(d):
        strata = np.floor(q[:, k] * n).astype(np.int64)
        np.testing.assert_array_equal(np.sort(strata), np.arange(n))
    if n >= 1000:
        assert not np.array_equal(np.argsort(q[:, 0]), np.argsort(q[:, 1]))


def test_native_lhs_shards_and_seeds(gpu):
    from probabilit_amd import native

    n = 200_000
    full = native.fill_lhs(5, n, 3)
    part = native.fill_lhs(5, n, 3, row0=70_000, nrows=50_000)
    np.testing.assert_array_equal(part, full[70_000:120_000])
    np.testing.assert_array_equal(native.fill_lhs(5, n, 3), full)
    assert not np.array_equal(native.fill_lhs(6, n, 3), full)


def test_native_uniform(gpu):
    from probabilit_amd import native

    q = native.fill_uniform(3, 1_000_000, 2)
    assert np.all((q >= 0) & (q < 1))
    assert abs(q.mean() - 0.5) < 2e-3
    assert abs(np.corrcoef(q.T)[0, 1]) < 5e-3


@pytest.mark.parametrize("name,kw", [("norm", {"loc": 1.11, "scale": 0.15}), ("lognorm", {"s": 0.5}),
                                     ("gamma", {"a": 2.0}), ("triang", {"c": 0.3}), ("poisson", {"mu": 4.0}),
                                     ("expon", {}), ("uniform", {"loc": -1.0, "scale": 3.0})])
def test_sobol_fused_ppf_equals_fill_then_ppf(gpu, name, kw):
    """pbh_sobol_ppf (the generator inside the inverse-CDF kernel, tail-compacted for norm /
    lognorm) gives exactly pbh_fill_sobol followed by pbh_ppf, for any row range."""
    import ctypes

    from probabilit_amd import _lib, device, native, qmc
    from probabilit_amd.modeling import _parse_scipy_args

    d, bits, col = 6, 30, 4
    sv, shift = qmc.sobol_setup(d, 5)
    svc, shc = np.ascontiguousarray(sv, np.uint32), np.ascontiguousarray(shift, np.uint32)
    for row0, n in [(0, 100_000), (12_345, 77_777)]:
        q = native.fill_sobol(sv, shift, n, row0=row0)[:, col]
        ref = native.ppf(name, q, **kw)
        params = [float(p) for p in _parse_scipy_args(name, (), kw)]
        arr = (_lib.Param * len(params))(*[_lib.Param(None, p) for p in params])
        out = device.empty(n)
        _lib.check(_lib.load().pbh_sobol_ppf(_lib.np_ptr(svc), _lib.np_ptr(shc), d, bits, row0, n, col,
                                             _lib.DIST_IDS[name], arr, len(params), out.data_ptr(), None,
                                             device.stream()), "pbh_sobol_ppf")
        np.testing.assert_array_equal(device.to_host(out), ref)


def test_sobol_dag_matches_materialised_quantiles(gpu):
    """A Sobol DAG (fused columns) equals sample_from_quantiles on the materialised points."""
    from probabilit_amd import native, qmc
    from probabilit_amd.modeling import Distribution

    def model():
        a = Distribution("norm", loc=1.0, scale=2.0)
        b = Distribution("gamma", a=2.0)
        c = Distribution("beta", a=2.0, b=3.0)  # no fused kernel: materialised column
        return a * b + c

    n = 4096
    y = model().sample(n, random_state=3, method="sobol")
    sv, shift = qmc.sobol_setup(3, 3)
    Q = native.fill_sobol(sv, shift, n)
    np.testing.assert_array_equal(y, model().sample_from_quantiles(Q))
