"""Inverse-CDF kernels vs the reference (scipy.stats ppf at modeling.py:807).

Gate: float results within rtol 1e-10 (north_star), discrete (poisson) results exact, NaN /
inf positions identical.  Golden values come from tests/golden/ppf.npz (reference run);
larger random sweeps compare against oracle.ppf (the same scipy call) on the box.
"""

import json
import zlib

import numpy as np
import pytest

from conftest import assert_close, golden

pytestmark = pytest.mark.gpu

RTOL = 1e-10

# scipy's poisson ppf is ceil(pdtrik(q, mu)) with a one-step pdtr correction; cdflib's root
# finder loses the answer when q underflows (< ~1e-160 for mu >= 1000) or q = 1 - 2^-53 for
# mu >= 2500, where it returns a k with pdtr(k, mu) < q.  The device kernel
# computes the defining quantity, the smallest k with pdtr(k, mu) >= q; outside this domain
# the test checks that definition instead of scipy's value.
POISSON_DOMAIN = (1e-150, 1.0 - 2.0**-52)


def _check_poisson(q, out, exp, mu, loc=0.0):
    import scipy.special as sc

    q = np.asarray(q)
    out = np.asarray(out) - loc
    exp = np.asarray(exp) - loc
    inside = (q >= POISSON_DOMAIN[0]) & (q <= POISSON_DOMAIN[1])
    np.testing.assert_array_equal(out[inside | ~np.isfinite(exp)], exp[inside | ~np.isfinite(exp)])
    mu = np.broadcast_to(mu, q.shape)
    for i in np.flatnonzero(~inside & np.isfinite(exp) & (q > 0) & (q < 1)):
        k = out[i]
        assert sc.pdtr(k, mu[i]) >= q[i] and (k == 0 or sc.pdtr(k - 1, mu[i]) < q[i]), (q[i], k)


@pytest.fixture(scope="module")
def ppf_golden():
    return golden("ppf.npz")


def _cases():
    z = golden("ppf.npz")
    return sorted(json.loads(str(z["meta"])).items())


@pytest.mark.parametrize("case", [c[0] for c in _cases()])
def test_ppf_golden(gpu, ppf_golden, case):
    from probabilit_amd import native

    name, kw = dict(_cases())[case]
    out = native.ppf(name, ppf_golden["q"], **kw)
    exp = ppf_golden[case]
    if name == "poisson":
        _check_poisson(ppf_golden["q"], out, exp, kw["mu"], kw.get("loc", 0.0))
    else:
        assert_close(out, exp, rtol=RTOL, what=case)


@pytest.mark.parametrize("dist,params", [
    ("norm", {"loc": "comp_loc", "scale": "comp_scale"}),
    ("poisson", {"mu": "comp_mu"}),
    ("gamma", {"a": "comp_a", "scale": "comp_scale"}),
    ("triang", {"c": "comp_c", "loc": "comp_loc", "scale": "comp_scale"}),
])
def test_ppf_composite_parameters(gpu, ppf_golden, dist, params):
    """Array-valued parameters: the composite broadcast of modeling.py:796-802."""
    from probabilit_amd import native

    kw = {k: ppf_golden[v] for k, v in params.items()}
    out = native.ppf(dist, ppf_golden["q"], **kw)
    exp = ppf_golden[f"comp_{dist}"]
    if dist == "poisson":
        _check_poisson(ppf_golden["q"], out, exp, kw["mu"])
    else:
        assert_close(out, exp, rtol=RTOL, what=dist)


@pytest.mark.parametrize("name,kw", [
    ("norm", {"loc": 2.0, "scale": 3.0}), ("gamma", {"a": 2.0}), ("gamma", {"a": 0.7, "scale": 3.0}),
    ("gamma", {"a": 0.05}), ("gamma", {"a": 45.0}), ("triang", {"c": 0.3}), ("expon", {"scale": 2.0}),
    ("lognorm", {"s": 1.3}), ("uniform", {"loc": 1.0, "scale": 2.0}),
    ("poisson", {"mu": 4.0}), ("poisson", {"mu": 30.0}), ("poisson", {"mu": 0.3}), ("poisson", {"mu": 2500.0}),
])
def test_ppf_random_sweep(gpu, name, kw):
    """2^18 random quantiles incl. extreme tails against the same scipy call."""
    from oracle.ppf import ppf as ref_ppf
    from probabilit_amd import native

    rng = np.random.default_rng(zlib.crc32(name.encode()))  # str hash() is salted per process
    q = np.concatenate([rng.random(2**18 - 4096), 10.0 ** rng.uniform(-300, -1, 2048),
                        1 - 10.0 ** rng.uniform(-16, -1, 2048)])
    out = native.ppf(name, q, **kw)
    exp = ref_ppf(name, q, **kw)
    if name == "poisson":
        _check_poisson(q, out, exp, kw["mu"])
    else:
        assert_close(out, exp, rtol=RTOL, what=f"{name}{kw}")


def test_fused_lhs_ppf_equals_two_pass(gpu):
    """pbh_lhs_ppf (q never stored) is bit-identical to pbh_fill_lhs + pbh_ppf."""
    from probabilit_amd import native

    n = 100_003
    for col, (name, kw) in enumerate([("norm", {}), ("gamma", {"a": 2.0}), ("poisson", {"mu": 4.0})]):
        fused = native.lhs_ppf(name, 1234, n, col, **kw)
        q = native.fill_lhs(1234, n, col + 1)[:, col]
        two = native.ppf(name, q, **kw)
        np.testing.assert_array_equal(fused, two)


def test_ppf_empty_and_nan(gpu):
    from probabilit_amd import native

    assert native.ppf("norm", np.zeros(0)).shape == (0,)
    out = native.ppf("gamma", np.array([np.nan, 0.0, 1.0, 0.5]), a=2.0)
    assert np.isnan(out[0]) and out[1] == 0.0 and np.isinf(out[2]) and np.isfinite(out[3])


@pytest.mark.parametrize("name,kw", [("triang", {"c": 0.3}), ("gamma", {"a": 2.0}), ("poisson", {"mu": 4.0}),
                                     ("expon", {}), ("norm", {"loc": 1.0, "scale": 2.0})])
def test_ppf_streaming_ragged_and_misaligned(gpu, name, kw):
    """k_ppf_v (contiguous, 16-byte aligned, 2048-draw tiles + a ragged end) and the plain k_ppf
    (taken for a column starting 8 bytes off) agree bit for bit, and with scipy."""
    import torch

    from oracle.ppf import ppf as ref_ppf
    from probabilit_amd import device, native

    rng = np.random.default_rng(11)
    qh = rng.random(3 * 2048 + 77)
    qd = torch.from_numpy(qh).to(device.device())
    for n in (1, 2047, 2048, 2049, 3 * 2048 + 76):
        aligned = native.ppf(name, qd[:n], **kw)   # offset 0: streaming kernel
        shifted = native.ppf(name, qd[1:n + 1], **kw)  # offset 8 B: plain kernel
        np.testing.assert_array_equal(aligned[1:], shifted[:n - 1])
        exp = ref_ppf(name, qh[:n], **kw)
        if name == "poisson":
            _check_poisson(qh[:n], aligned, exp, kw["mu"])
        else:
            assert_close(aligned, exp, rtol=RTOL, what=f"{name}{kw} n={n}")


@pytest.mark.parametrize("kw", [{"a": 2.0}, {"a": 0.7, "scale": 3.0}, {"a": 0.05}, {"a": 45.0, "loc": 1.0}])
def test_gamma_lds_table_bit_identical(gpu, kw):
    """k_ppf_gamma_lds / k_lhs_ppf_gamma_lds (guide table staged in LDS; scalar parameters) give
    the same bits as k_ppf / k_lhs_ppf reading the table from global memory (taken when loc is
    a per-row vector, here all equal to the scalar) and as the stratum-ordered generator."""
    import ctypes

    from probabilit_amd import _lib, device, native

    n = 200_003
    lds = native.lhs_ppf("gamma", 99, n, 3, **kw)
    vec = dict(kw, loc=np.full(n, kw.get("loc", 0.0)))
    glob = native.lhs_ppf("gamma", 99, n, 3, **vec)
    np.testing.assert_array_equal(lds, glob)
    q = native.fill_lhs(99, n, 4)[:, 3]
    np.testing.assert_array_equal(native.ppf("gamma", q, **kw), native.ppf("gamma", q, **vec))
    np.testing.assert_array_equal(native.ppf("gamma", q, **kw), lds)
    out, flag = device.empty(n), device.zeros(1, "int32")
    prm = (ctypes.c_double * 3)(kw["a"], kw.get("loc", 0.0), kw.get("scale", 1.0))
    _lib.check(_lib.load().pbh_lhs_sorted_ppf(99, n, 0, n, 3, _lib.DIST_IDS["gamma"], prm, 3, out.data_ptr(),
                                              flag.data_ptr(), device.stream()), "pbh_lhs_sorted_ppf")
    np.testing.assert_array_equal(np.sort(lds), np.sort(device.to_host(out)))


@pytest.mark.parametrize("kw", [{"mu": 4.0}, {"mu": 30.0}, {"mu": 0.3, "loc": 2.0}, {"mu": 2500.0}, {"mu": 1e5}])
def test_poisson_lds_table_bit_identical(gpu, kw):
    """k_ppf_poisson_lds / k_lhs_ppf_poisson_lds (CDF table + guide staged in LDS; scalar mu and
    loc, tables up to 6144 entries -- mu = 1e5 takes the global-table kernel) agree exactly with
    the global-table kernels (taken for a per-row loc) and with scipy inside its domain."""
    from oracle.ppf import ppf as ref_ppf
    from probabilit_amd import native

    n = 200_003
    vec = dict(kw, loc=np.full(n, kw.get("loc", 0.0)))
    lds = native.lhs_ppf("poisson", 5, n, 1, **kw)
    np.testing.assert_array_equal(lds, native.lhs_ppf("poisson", 5, n, 1, **vec))
    q = native.fill_lhs(5, n, 2)[:, 1]
    out = native.ppf("poisson", q, **kw)
    np.testing.assert_array_equal(out, native.ppf("poisson", q, **vec))
    np.testing.assert_array_equal(out, lds)
    _check_poisson(q[:20000], out[:20000], ref_ppf("poisson", q[:20000], **kw), kw["mu"], kw.get("loc", 0.0))
