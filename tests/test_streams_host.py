"""CPU check of the MT19937 jump-ahead and PCG64 advance algebra of pbh_mt.h (compiled for
the host by tests/native/streams_host.cpp) against numpy's own bit generators -- the
generators behind check_random_state(...).random at modeling.py:484-486 and behind
scipy.stats.qmc.LatinHypercube (modeling.py:480,488)."""

import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "streams_host.cpp")
OUT = os.path.join(HERE, "native", "_build", "libpbh_streams_host.so")


@pytest.fixture(scope="module")
def sh():
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    if hipcc is None:
        pytest.skip("hipcc not available")
    deps = [SRC] + [os.path.join(ROOT, "probabilit_amd", "csrc", f) for f in ("pbh_mt.h", "pbh_common.h", "pbh_rng.h")]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "-I", os.path.join(ROOT, "probabilit_amd", "csrc"),
                        "-I", os.path.join(ROOT, "include"), SRC, "-o", OUT], check=True, capture_output=True)
    return ctypes.CDLL(OUT)


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _mt_state(rs):
    st = rs.get_state(legacy=False)["state"]
    return np.ascontiguousarray(st["key"], dtype=np.uint32), int(st["pos"])


def _raw(key, pos, count):
    bg = np.random.MT19937()
    bg.state = {"bit_generator": "MT19937", "state": {"key": key, "pos": pos}}
    return bg.random_raw(count).astype(np.uint32)


def test_charpoly_degree(sh):
    phi = np.zeros(312, np.uint64)
    assert sh.sh_mt_charpoly(_p(phi)) == 0
    assert int(phi[311]) >> 33 == 1 and int(phi[0]) & 1 == 1  # monic of degree 19937, phi(0) = 1


@pytest.mark.parametrize("seed", [0, 1, 12345])
@pytest.mark.parametrize("offset,count", [(0, 700), (1, 5), (623, 3), (624, 10), (12345, 100), (1_999_000, 1000)])
def test_mt_jump_matches_numpy(sh, seed, offset, count):
    key, pos = _mt_state(np.random.RandomState(seed))
    raw = _raw(key, pos, offset + count)  # words pos + 0 .. of the key sequence
    out = np.zeros(count, np.uint32)
    assert sh.sh_mt_words(_p(key), ctypes.c_int64(pos + offset), ctypes.c_int64(count), _p(out)) == 0
    np.testing.assert_array_equal(out, raw[offset:])


def test_mt_jump_mid_block_state(sh):
    rs = np.random.RandomState(7)
    rs.random(333)  # pos mid-block
    key, pos = _mt_state(rs)
    assert 0 < pos < 624
    raw = _raw(key, pos, 5000)
    out = np.zeros(4000, np.uint32)
    assert sh.sh_mt_words(_p(key), ctypes.c_int64(pos + 1000), ctypes.c_int64(4000), _p(out)) == 0
    np.testing.assert_array_equal(out, raw[1000:])


@pytest.mark.parametrize("seed", [0, 42])
def test_pcg64_advance_and_doubles(sh, seed):
    g = np.random.default_rng(seed)
    st = g.bit_generator.state["state"]
    s, inc = st["state"], st["inc"]
    M = (1 << 64) - 1
    ref = g.random(5000)
    out = np.zeros(1000, np.float64)
    sh.sh_pcg_doubles(ctypes.c_uint64(s & M), ctypes.c_uint64(s >> 64), ctypes.c_uint64(inc & M),
                      ctypes.c_uint64(inc >> 64), ctypes.c_uint64(4000), ctypes.c_int64(1000), _p(out))
    np.testing.assert_array_equal(out, ref[4000:])
    adv = np.zeros(2, np.uint64)
    sh.sh_pcg_advance(ctypes.c_uint64(s & M), ctypes.c_uint64(s >> 64), ctypes.c_uint64(inc & M),
                      ctypes.c_uint64(inc >> 64), ctypes.c_uint64(5000), _p(adv))
    assert int(adv[0]) | (int(adv[1]) << 64) == g.bit_generator.state["state"]["state"]


def test_pcg64_advance_python():
    from probabilit_amd.qmc import pcg64_advance

    g = np.random.default_rng(3)
    st = g.bit_generator.state["state"]
    g.random(12345)
    assert pcg64_advance(st["state"], st["inc"], 12345) == g.bit_generator.state["state"]["state"]


def test_check_random_state_semantics():
    from probabilit_amd.qmc import check_random_state

    assert check_random_state(None) is np.random.mtrand._rand
    assert isinstance(check_random_state(3), np.random.RandomState)
    g = np.random.default_rng(1)
    assert check_random_state(g) is g
    with pytest.raises(ValueError):
        check_random_state("x")


# ---------------------------------------------------------------- reference LHS shuffles (host half)
@pytest.mark.parametrize("n,d,seed,draws", [(1, 1, 0, 0), (7, 5, 9, 0), (4096, 8, 0, 0), (100_000, 32, 3, 5),
                                            (20_001, 1, 4, 1)])
def test_lhs_reference_perms_match_numpy_shuffle(n, d, seed, draws):
    """pbh_lhs_reference_perms (host C++, the sequential half of the reference LHS stream)
    against numpy's Generator.shuffle on the same PCG64 state, LatinHypercube._random_lhs's
    d shuffles of arange(1, n + 1) after rng.uniform(size=(n, d)); the final state (with the
    buffered 32-bit half) must match too.  `draws` 32-bit draws first leave a buffered half."""
    from probabilit_amd import _lib, qmc

    lib = _lib.load()  # host-only entry point: no GPU is touched
    g = np.random.default_rng(seed)
    g.integers(0, 2, size=draws, dtype=np.uint32)
    g.uniform(size=(n, d))
    st = g.bit_generator.state
    ref = np.tile(np.arange(1, n + 1), (d, 1))
    for i in range(d):
        g.shuffle(ref[i])
    out = np.empty((d, n), dtype=np.int32)
    so = np.zeros(4, dtype=np.uint64)
    sw, iw = qmc._u128_words(st["state"]["state"]), qmc._u128_words(st["state"]["inc"])
    _lib.check(lib.pbh_lhs_reference_perms(_lib.np_ptr(sw), _lib.np_ptr(iw), st["has_uint32"], st["uinteger"], n, d,
                                           _lib.np_ptr(out), _lib.np_ptr(so)))
    np.testing.assert_array_equal(out, ref)
    end = g.bit_generator.state
    assert (int(so[0]) | (int(so[1]) << 64)) == end["state"]["state"]
    assert (int(so[2]), int(so[3])) == (end["has_uint32"], end["uinteger"])


def test_lhs_reference_perms_vs_oracle_restatement():
    """The same host half against the oracle's pure-Python restatement of _random_lhs
    (oracle/streams.py lhs_reference), which tests/test_oracle.py pins to the golden LHS."""
    from oracle import streams
    from probabilit_amd import _lib, qmc

    lib = _lib.load()
    n, d = 300, 4
    eng = qmc.engine_rng(5)
    st = eng.bit_generator.state
    s, inc = int(st["state"]["state"]), int(st["state"]["inc"])
    q = streams.lhs_reference((s, inc), n, d)
    out = np.empty((d, n), dtype=np.int32)
    sw, iw = qmc._u128_words(qmc.pcg64_advance(s, inc, n * d)), qmc._u128_words(inc)
    _lib.check(lib.pbh_lhs_reference_perms(_lib.np_ptr(sw), _lib.np_ptr(iw), 0, 0, n, d, _lib.np_ptr(out), None))
    np.testing.assert_array_equal(out.T, np.ceil(q * n).astype(np.int64))


def test_native_lhs_statistics(sh):
    """The native LHS design (pbh_rng.h: 4-round keyed FE2 Feistel stratum + SplitMix64 jitter),
    host-compiled: every column is a Latin hypercube column, and at n = 1e6 the Spearman
    correlations between columns, with the row index, and between consecutive rows are those of
    independent random permutations (|rho| < 5 / sqrt(n)); the in-stratum jitter is uniform
    (Kolmogorov-Smirnov)."""
    import scipy.stats

    n, d = 1_000_000, 8
    q = np.empty(n * d)
    sh.sh_native_lhs(ctypes.c_uint64(1234), ctypes.c_int64(n), 0, d, _p(q))
    q = q.reshape(d, n)
    strata = np.floor(q * n).astype(np.int64)
    bound = 5.0 / np.sqrt(n)
    rows = np.arange(n)
    for c in range(d):
        assert np.array_equal(np.sort(strata[c]), rows), f"column {c} is not a Latin hypercube column"
        assert abs(np.corrcoef(strata[c], rows)[0, 1]) < bound
        assert abs(np.corrcoef(strata[c][:-1], strata[c][1:])[0, 1]) < bound
        for c2 in range(c):
            assert abs(np.corrcoef(strata[c], strata[c2])[0, 1]) < bound, (c, c2)
    jitter = (q * n - strata).ravel()
    assert scipy.stats.kstest(jitter, "uniform").pvalue > 1e-4
