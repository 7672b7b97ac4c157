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
    deps = [SRC] + [os.path.join(ROOT, "probabilit_amd", "csrc", f) for f in ("pbh_mt.h", "pbh_common.h")]
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
