"""numpy's bit-generator streams on the GPU, bit for bit (modeling.py:484-486).

method=None draws check_random_state(random_state).random((size, d)): an int or None gives a
RandomState (MT19937, pbh_mt19937_random), a Generator gives PCG64 (pbh_pcg64_random).  The
oracle here is numpy itself (the reference's own generator) plus the golden draws the
reference produced (tests/golden/streams.npz mt_s0_999x1) and the docstring pins of
modeling.py:443-449.
"""

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


def _src_matrix(src):
    from probabilit_amd import device

    cols = [device.to_host(src.column(c)[1]) for c in range(src.d)]
    return np.column_stack(cols) if cols else np.empty((src.rows, 0))


@pytest.mark.parametrize("seed", [0, 1, 2**32 - 1])
@pytest.mark.parametrize("n,d", [(1, 1), (999, 1), (1000, 3), (4099, 32), (300_001, 7)])
def test_mt19937_matches_randomstate(gpu, seed, n, d):
    from probabilit_amd import qmc

    src = qmc.pseudo_random_source(n, d, seed)
    np.testing.assert_array_equal(_src_matrix(src), np.random.RandomState(seed).random((n, d)))


def test_mt19937_large_segments(gpu):
    """Several jump-ahead segments (2 n d = 1.6e7 words)."""
    from probabilit_amd import qmc

    n, d = 1_000_000, 8
    src = qmc.pseudo_random_source(n, d, 11)
    q = _src_matrix(src)
    ref = np.random.RandomState(11).random((n, d))
    np.testing.assert_array_equal(q, ref)


def test_mt19937_golden_cfg1(gpu):
    from probabilit_amd import qmc

    z = golden("streams.npz")
    np.testing.assert_array_equal(_src_matrix(qmc.pseudo_random_source(999, 1, 0)), z["mt_s0_999x1"])


@pytest.mark.parametrize("draws_before", [0, 1, 333, 623, 624, 5000])
def test_mt19937_state_writeback(gpu, draws_before):
    """A caller's RandomState (any pos) yields numpy's draws and ends in numpy's state."""
    from probabilit_amd import qmc

    rs, ref = np.random.RandomState(5), np.random.RandomState(5)
    rs.random(draws_before)
    ref.random(draws_before)
    src = qmc.pseudo_random_source(777, 3, rs)
    np.testing.assert_array_equal(_src_matrix(src), ref.random((777, 3)))
    a, b = rs.get_state(legacy=False), ref.get_state(legacy=False)
    assert a["state"]["pos"] == b["state"]["pos"]
    np.testing.assert_array_equal(a["state"]["key"], b["state"]["key"])
    np.testing.assert_array_equal(rs.random(1000), ref.random(1000))


def test_mt19937_global_state(gpu):
    from probabilit_amd import qmc

    np.random.seed(123)
    src = qmc.pseudo_random_source(50, 2, None)
    q = _src_matrix(src)
    np.random.seed(123)
    np.testing.assert_array_equal(q, np.random.random((50, 2)))
    after = np.random.random(10)
    np.random.seed(123)
    np.random.random((50, 2))
    np.testing.assert_array_equal(after, np.random.random(10))


def test_mt19937_row_shard(gpu):
    from probabilit_amd import qmc

    src = qmc.pseudo_random_source(10_000, 5, 9).shard(3001, 4000)
    ref = np.random.RandomState(9).random((10_000, 5))[3001:7001]
    np.testing.assert_array_equal(_src_matrix(src), ref)


@pytest.mark.parametrize("n,d", [(1, 1), (1000, 3), (100_003, 32)])
def test_pcg64_generator(gpu, n, d):
    from probabilit_amd import qmc

    g, ref = np.random.default_rng(17), np.random.default_rng(17)
    g.integers(0, 10, size=3, dtype=np.uint32)  # leave a buffered 32-bit half behind
    ref.integers(0, 10, size=3, dtype=np.uint32)
    src = qmc.pseudo_random_source(n, d, g)
    np.testing.assert_array_equal(_src_matrix(src), ref.random((n, d)))
    assert g.bit_generator.state == ref.bit_generator.state
    np.testing.assert_array_equal(g.integers(0, 1 << 30, size=5), ref.integers(0, 1 << 30, size=5))


def test_docstring_pins_pseudo_random(gpu):
    """modeling.py:443-447."""
    from probabilit_amd.modeling import Distribution

    result = 2 * Distribution("expon", scale=1 / 3)
    np.testing.assert_allclose(result.sample(random_state=0), [0.53058301], rtol=1e-8)
    np.testing.assert_allclose(result.sample(size=5, random_state=0),
                               [0.53058301, 0.83728718, 0.6154821, 0.52480077, 0.36736566], rtol=1e-7)


def test_cfg1_readme_norm(gpu):
    """BASELINE config 1: Distribution("norm", loc=176, scale=7.1).sample(999, random_state=0)
    equals scipy's norm.ppf of RandomState(0).random((999, 1)) (the reference's computation)."""
    import scipy.stats

    from probabilit_amd.modeling import Distribution

    x = Distribution("norm", loc=176, scale=7.1).sample(999, random_state=0)
    ref = scipy.stats.norm(loc=176, scale=7.1).ppf(np.random.RandomState(0).random((999, 1))[:, 0])
    np.testing.assert_allclose(x, ref, rtol=1e-10, atol=0)


@pytest.mark.parametrize("d,seed,n", [(1, 0, 10), (5, 0, 1000), (12, 3, 4097), (32, 123, 20_000)])
def test_halton_matches_scipy(gpu, d, seed, n):
    import scipy.stats

    from probabilit_amd import qmc

    src = qmc.make_source("halton", n, d, seed)
    np.testing.assert_array_equal(_src_matrix(src), scipy.stats.qmc.Halton(d, rng=seed).random(n))


def test_halton_row_shard_and_large_index(gpu):
    """Shards regenerate any index range; indices past 2^32 take the 64-bit digit path."""
    from scipy.stats._qmc import van_der_corput

    from probabilit_amd import device, qmc

    src = qmc.make_source("halton", 2**32 + 200, 3, 7).shard(2**32 + 5, 100)
    q = _src_matrix(src)
    perms = np.split(src.perms, np.cumsum(src.counts * src.bases)[:-1])
    for c, b in enumerate(src.bases):
        ref = van_der_corput(100, int(b), start_index=2**32 + 5, scramble=True,
                             permutations=perms[c].reshape(src.counts[c], b))
        np.testing.assert_array_equal(q[:, c], ref)
    del device


def test_halton_node_sample(gpu):
    """Node.sample(method="halton") equals the reference's computation: scipy Halton quantiles
    (modeling.py:481,488) through the ppf (modeling.py:807)."""
    import scipy.stats

    from probabilit_amd.modeling import Distribution

    a, b = Distribution("norm", loc=1, scale=2), Distribution("expon", scale=3)
    out = (a * b).sample(513, random_state=4, method="halton")
    Q = scipy.stats.qmc.Halton(2, rng=4).random(513)
    ref = scipy.stats.norm(1, 2).ppf(Q[:, 0]) * scipy.stats.expon(scale=3).ppf(Q[:, 1])
    np.testing.assert_allclose(out, ref, rtol=1e-10)


# ---------------------------------------------------------------- reference LHS stream (row a2)
@pytest.mark.parametrize("key,d,seed,n", [("lhs_d8_s0_n4096", 8, 0, 4096), ("lhs_d3_s123_n1000", 3, 123, 1000)])
def test_reference_lhs_matches_golden(gpu, key, d, seed, n):
    """stream="reference": LatinHypercube(d, rng=seed).random(n) bit for bit, against the
    vectors the reference's scipy produced (tests/golden/make_golden.py)."""
    from probabilit_amd import qmc

    src = qmc.make_source("lhs", n, d, seed, stream="reference")
    np.testing.assert_array_equal(_src_matrix(src), golden("streams.npz")[key])


@pytest.mark.parametrize("n,d,seed", [(1, 1, 0), (2, 3, 5), (50_000, 32, 9), (1_000_003, 4, 2)])
def test_reference_lhs_matches_scipy(gpu, n, d, seed):
    import scipy.stats

    from probabilit_amd import qmc

    src = qmc.make_source("lhs", n, d, seed, stream="reference")
    np.testing.assert_array_equal(_src_matrix(src), scipy.stats.qmc.LatinHypercube(d=d, rng=seed).random(n))


def test_reference_lhs_generator_spawn(gpu):
    """A Generator passed as random_state is used the way scipy uses it (an owned child is
    spawned from it), so the caller's generator ends in the same state as under scipy."""
    import scipy.stats

    from probabilit_amd import qmc

    g, ref = np.random.default_rng(21), np.random.default_rng(21)
    q = _src_matrix(qmc.make_source("lhs", 777, 5, g, stream="reference"))
    np.testing.assert_array_equal(q, scipy.stats.qmc.LatinHypercube(d=5, rng=ref).random(777))
    np.testing.assert_array_equal(g.random(4), ref.random(4))


def test_docstring_pin_lhs_reference_stream(gpu):
    """modeling.py:448-449: result.sample(size=5, random_state=0, method="lhs")."""
    from probabilit_amd.modeling import Distribution

    result = 2 * Distribution("expon", scale=1 / 3)
    out = result.sample(size=5, random_state=0, method="lhs", stream="reference")
    # the doctest shows numpy's 8-decimal repr: agreement to half a unit in the 8th decimal
    np.testing.assert_allclose(out, [1.11212876, 0.273718, 0.03808862, 0.5702549, 0.83779147], rtol=0, atol=5e-9)
    # and the exact value: scipy's LatinHypercube quantiles through scipy's expon ppf, times 2
    import scipy.stats

    q = scipy.stats.qmc.LatinHypercube(d=1, rng=0).random(5)[:, 0]
    np.testing.assert_allclose(out, 2 * scipy.stats.expon(scale=1 / 3).ppf(q), rtol=1e-10, atol=0)


def test_reference_lhs_module_default(gpu):
    from probabilit_amd import qmc
    from probabilit_amd.modeling import Distribution

    x = Distribution("norm")
    native = x.sample(100, random_state=3, method="lhs").copy()
    qmc.set_default_stream("reference")
    try:
        ref = x.sample(100, random_state=3, method="lhs")
    finally:
        qmc.set_default_stream("native")
    import scipy.stats

    q = scipy.stats.qmc.LatinHypercube(d=1, rng=3).random(100)[:, 0]
    np.testing.assert_allclose(ref, scipy.stats.norm.ppf(q), rtol=1e-10, atol=0)
    assert not np.array_equal(native, ref)
    np.testing.assert_array_equal(x.sample(100, random_state=3, method="lhs"), native)


def test_reference_lhs_correlated_dag_matches_reference_pipeline(gpu):
    """The cfg3 graph (d=32) on the reference stream: the whole reference computation
    (scipy LHS -> scipy ppf -> Iman-Conover, oracle.pipeline) on the same seed, values
    within 1e-10 and identical ranks (a rank difference moves a value by a whole spacing)."""
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, lhs_quantiles, ppf_columns
    from probabilit_amd.modeling import Distribution, NoOp

    from conftest import assert_close

    n, d, seed = 20_000, 32, 11
    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    C = cfg3_corr(d)
    NoOp(*ds).correlate(*ds, corr_mat=C).sample(n, random_state=seed, method="lhs", stream="reference")
    Y = np.column_stack([x.samples_ for x in ds])
    ref = oic.iman_conover(ppf_columns(lhs_quantiles(n, d, seed), cfg_dists(d)), C)["Y"]
    assert_close(Y, ref, rtol=1e-10, what="reference-stream cfg3 DAG vs the reference pipeline")


def _ref_stats():
    import ctypes

    from probabilit_amd import _lib

    dev, att, amb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    _lib.check(_lib.load().pbh_lhs_reference_stats(ctypes.byref(dev), ctypes.byref(att), ctypes.byref(amb)))
    return dev.value, att.value, amb.value


def _ref_lhs_direct(state, inc, has32, buf32, n, d):
    """pbh_lhs_reference at an arbitrary PCG64 state (has32 / buf32 included)."""
    import ctypes

    from probabilit_amd import _lib, device
    from probabilit_amd.qmc import _u128_words

    lib = _lib.load()
    nb = ctypes.c_size_t()
    _lib.check(lib.pbh_lhs_reference_workspace_size(n, d, ctypes.byref(nb)))
    ws = device.empty(int(nb.value), "uint8")
    q = device.empty((d, n))
    s, i = _u128_words(state), _u128_words(inc)
    _lib.check(lib.pbh_lhs_reference(_lib.np_ptr(s), _lib.np_ptr(i), has32, buf32, n, d, q.data_ptr(), n,
                                     ws.data_ptr(), ws.numel(), device.stream()), "pbh_lhs_reference")
    return device.to_host(q).T


def _ref_lhs_host(state, inc, has32, buf32, n, d):
    """The same matrix from the host shuffles (pbh_lhs_reference_perms, pinned against numpy's
    Generator.shuffle in test_streams_host.py) and numpy's own uniforms."""
    import ctypes

    from probabilit_amd import _lib
    from probabilit_amd.qmc import _u128_words

    g = np.random.Generator(np.random.PCG64())
    g.bit_generator.state = {"bit_generator": "PCG64", "state": {"state": state, "inc": inc},
                             "has_uint32": has32, "uinteger": buf32}
    u = g.uniform(size=(n, d))
    st = g.bit_generator.state
    perms = np.empty((d, n), dtype=np.int32)
    s, i = _u128_words(st["state"]["state"]), _u128_words(inc)
    _lib.check(_lib.load().pbh_lhs_reference_perms(_lib.np_ptr(s), _lib.np_ptr(i), has32, buf32, n, d,
                                                   _lib.np_ptr(perms), None))
    return (perms.T - u) / n


@pytest.mark.parametrize("n,d,has32", [(2, 3, 0), (3, 5, 1), (1000, 4, 1), (65_537, 3, 0), (1_000_003, 4, 1),
                                       (3_000_000, 2, 0)])
def test_reference_lhs_device_decode(gpu, n, d, has32):
    """The shuffles decoded on the device (pbh_lhs_dev.hip: banded classification, host walk of
    the ambiguous draws, every decision re-checked) equal the host shuffles bit for bit, from an
    arbitrary PCG64 state with and without numpy's buffered 32-bit half, in one attempt."""
    rng = np.random.default_rng(n + d)
    state, inc = int(rng.integers(0, 2**63)) << 64 | int(rng.integers(0, 2**63)), (int(rng.integers(0, 2**62)) << 1) | 1
    buf32 = int(rng.integers(0, 2**32)) if has32 else 0
    got = _ref_lhs_direct(state, inc, has32, buf32, n, d)
    dev, att, amb = _ref_stats()
    np.testing.assert_array_equal(got, _ref_lhs_host(state, inc, has32, buf32, n, d))
    assert dev == 1 and att == 1, (dev, att, amb)
    print(f"n={n} d={d}: ambiguous draws walked on the host {amb} ({amb / d:.0f} per column)")


def test_reference_lhs_device_decode_retry_and_fallback(gpu):
    """A band too narrow for the walk fails the device check: the call retries with wider bands,
    then falls back to the host shuffles; the result is the same matrix either way."""
    import ctypes

    from probabilit_amd import _lib

    lib = _lib.load()
    n, d, seed = 200_000, 3, 4
    import scipy.stats

    ref = scipy.stats.qmc.LatinHypercube(d=d, rng=seed).random(n)
    from probabilit_amd import qmc

    prev = ctypes.c_double()
    _lib.check(lib.pbh_lhs_reference_band(1e-3, ctypes.byref(prev)))
    try:
        got = _src_matrix(qmc.make_source("lhs", n, d, seed, stream="reference"))
        dev, att, amb = _ref_stats()
    finally:
        _lib.check(lib.pbh_lhs_reference_band(prev.value, None))
    np.testing.assert_array_equal(got, ref)
    assert att == 3 and dev == 0, (dev, att, amb)
    got = _src_matrix(qmc.make_source("lhs", n, d, seed, stream="reference"))
    np.testing.assert_array_equal(got, ref)
    assert _ref_stats()[:2] == (1, 1)


def _ref_lhs_strata(state, inc, has32, buf32, n, d):
    """pbh_lhs_reference_strata: the matrix and each row's stratum."""
    import ctypes

    from probabilit_amd import _lib, device
    from probabilit_amd.qmc import _u128_words

    lib = _lib.load()
    nb = ctypes.c_size_t()
    _lib.check(lib.pbh_lhs_reference_workspace_size(n, d, ctypes.byref(nb)))
    ws = device.empty(int(nb.value), "uint8")
    q, t = device.empty((d, n)), device.empty((d, n), "int32")
    s, i = _u128_words(state), _u128_words(inc)
    _lib.check(lib.pbh_lhs_reference_strata(_lib.np_ptr(s), _lib.np_ptr(i), has32, buf32, n, d, q.data_ptr(), n,
                                            t.data_ptr(), n, ws.data_ptr(), ws.numel(), device.stream()),
               "pbh_lhs_reference_strata")
    return device.to_host(q).T, device.to_host(t).T


@pytest.mark.parametrize("narrow", [False, True])
def test_reference_lhs_strata(gpu, narrow):
    """The strata beside the matrix (device decode, and the host-shuffle fallback a too-narrow
    band forces): perms - 1 of the host shuffles, so every q lies in its stratum's interval."""
    import ctypes

    from probabilit_amd import _lib

    n, d, has32 = 100_003, 3, 1
    rng = np.random.default_rng(5)
    state, inc = int(rng.integers(0, 2**63)) << 64 | int(rng.integers(0, 2**63)), (int(rng.integers(0, 2**62)) << 1) | 1
    buf32 = int(rng.integers(0, 2**32))
    lib = _lib.load()
    prev = ctypes.c_double()
    _lib.check(lib.pbh_lhs_reference_band(1e-3 if narrow else 0.0, ctypes.byref(prev)))
    try:
        q, t = _ref_lhs_strata(state, inc, has32, buf32, n, d)
        dev = _ref_stats()[0]
    finally:
        _lib.check(lib.pbh_lhs_reference_band(prev.value, None))
    assert dev == (0 if narrow else 1)
    np.testing.assert_array_equal(q, _ref_lhs_host(state, inc, has32, buf32, n, d))
    np.testing.assert_array_equal(np.sort(t, axis=0), np.tile(np.arange(n, dtype=np.int32)[:, None], (1, d)))
    assert np.all(q > t / n) and np.all(q <= (t + 1) / n)


def test_iman_conover_strata_equals_sort(gpu):
    """Iman-Conover given the columns' strata (step 1 by scatter, certified on the device) equals
    Iman-Conover sorting them: Y, the scores and E identical.  Covered: continuous columns,
    discrete ones (ties: average ranks from the runs), and hints the check must reject (a
    decreasing transform of the column, strata that are not a permutation): those columns are
    sorted instead, with the same result."""
    import scipy.stats

    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd import device, qmc
    from probabilit_amd.correlation import ImanConover

    n, d, seed = 50_000, 8, 7
    src = qmc.make_source("lhs", n, d, seed, stream="reference")
    src.keep_strata = True
    q = device.to_host(src.matrix())
    strata = [src.strata_of(c) for c in range(d)]
    dists = cfg_dists(d)
    X = np.stack([getattr(scipy.stats, nm)(**kw).ppf(q[c]) for c, (nm, kw) in enumerate(dists)])
    X[5] = -X[5]  # decreasing: the strata are not its ranks (inversions) -> sorted
    bad = device.to_host(strata[6]).copy()
    bad[10] = bad[11]  # not a permutation: a stratum left NaN -> sorted
    strata[6] = device.to_device(bad)
    strata[7] = None  # no hint
    block = device.to_device(X).contiguous()
    ic = ImanConover().set_target(cfg3_corr(d))
    dbg_a = {"S": device.empty((d, n)), "E": np.zeros((d, d))}
    dbg_b = {"S": device.empty((d, n)), "E": np.zeros((d, d))}
    Ya = device.to_host(ic._transform_device(block, strata=strata, debug=dbg_a))
    Yb = device.to_host(ic._transform_device(block, debug=dbg_b))
    np.testing.assert_array_equal(device.to_host(dbg_a["S"]), device.to_host(dbg_b["S"]))
    np.testing.assert_array_equal(dbg_a["E"], dbg_b["E"])
    np.testing.assert_array_equal(Ya, Yb)
    assert any(nm == "poisson" for nm, _ in dists)  # a tied column took the heads branch
