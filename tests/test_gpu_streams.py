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
