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

# scipy's poisson ppf is ceil(pdtrik(q, mu)) with a one-step pdtr correction; the device
# reproduces it bit for bit: the definition from its CDF table, and cdflib's search restated in
# pbh_cdflib.h (with glibc's exp / log, pbh_glibc.h) inside the window above each CDF value and
# below 1e-150, where scipy's own answer departs from the definition.  No allowance.
def _check_poisson(q, out, exp, mu, loc=0.0):
    np.testing.assert_array_equal(np.asarray(out), np.asarray(exp))


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
    """pbh_lhs_ppf (q never stored) is bit-identical to pbh_fill_lhs + pbh_ppf, for the base
    set and the pbh_ppf_ext distributions (the LHS quantile generated inside k_ppf_ext), with a
    row offset too."""
    from probabilit_amd import native

    n = 100_003
    for col, (name, kw) in enumerate([("norm", {}), ("gamma", {"a": 2.0}), ("poisson", {"mu": 4.0}),
                                      ("beta", {"a": 3.4, "b": 2.6}), ("binom", {"n": 20, "p": 0.3}),
                                      ("weibull_min", {"c": 1.5}), ("loguniform", {"a": 0.5, "b": 8.0}),
                                      ("chi2", {"df": 3.0})]):
        fused = native.lhs_ppf(name, 1234, n, col, **kw)
        q = native.fill_lhs(1234, n, col + 1)[:, col]
        two = native.ppf(name, q, **kw)
        np.testing.assert_array_equal(fused, two)
        np.testing.assert_array_equal(native.lhs_ppf(name, 1234, n, col, row0=777, nrows=5000, **kw), two[777:5777])


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


# ---------------------------------------------------------------- dense parity at the bench parameters
def _sorted_column(seed, n, col, name, kw):
    """k_lhs_sorted_ppf's output (the stratum-ordered generator the bench runs) and the sorted
    native quantiles of the same column (stratum t holds the t-th smallest quantile)."""
    import ctypes

    import torch

    from probabilit_amd import _lib, device
    from probabilit_amd.modeling import _parse_scipy_args

    params = [float(v) for v in _parse_scipy_args(name, (), kw)]
    out, flag = device.empty(n), device.zeros(1, "int32")
    prm = (ctypes.c_double * 3)(*params)
    lib = _lib.load()
    _lib.check(lib.pbh_lhs_sorted_ppf(seed, n, 0, n, col, _lib.DIST_IDS[name], prm, len(params), out.data_ptr(),
                                      flag.data_ptr(), device.stream()), "pbh_lhs_sorted_ppf")
    q = device.empty(n)
    _lib.check(lib.pbh_fill_lhs(seed, n, 0, n, col, 1, q.data_ptr(), n, device.stream()), "pbh_fill_lhs")
    q = torch.sort(q).values
    return device.to_host(out), device.to_host(q)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("col,name,kw", [(1, "gamma", {"a": 2.0}), (5, "gamma", {"a": 0.7, "scale": 3.0}),
                                         (3, "poisson", {"mu": 4.0}), (7, "poisson", {"mu": 30.0})])
def test_stratum_generator_dense_vs_scipy_1e7(gpu, col, name, kw):
    """Every stratum value of a native-LHS column at N = 1e7 from the stratum-ordered generator
    (k_lhs_sorted_ppf: the bench's step-1 kernel, guided igami / CDF table) against
    scipy.stats.<dist>.ppf of the same quantiles: continuous within 1e-10
    relative, discrete exact."""
    from oracle.pipeline import ppf_columns

    n = 10_000_000
    x, q = _sorted_column(2024, n, col, name, kw)
    exp = ppf_columns(q[:, None], [(name, kw)], threads=16)[:, 0]
    if name == "poisson":
        np.testing.assert_array_equal(x, exp)
    else:
        bad = int(np.count_nonzero(np.abs(x - exp) > RTOL * np.abs(exp)))
        assert bad == 0, f"{bad} of {n} stratum values beyond rtol {RTOL}"


@pytest.mark.parametrize("a", [0.05, 0.1, 0.3, 0.7, 1.0, 2.0, 3.5, 10.0, 45.0, 250.0, 3000.0, 1e5])
def test_gamma_guide_every_interval(gpu, a):
    """The guided igami at every interval of the per-parameter guide grid (w_j = -80 + j / 32,
    j < 3841, pbh_special.h): both endpoints, the quarter points and the midpoint of each
    interval, plus w one ulp either side of each node, mapped to p = 1 / (1 + e^-w) (and
    through the complement above w = 0), against scipy's gammaincinv at 1e-10 relative --
    the interpolant's error bound is checked per interval only at the midpoint when the
    table is built, so this covers the rest of each interval."""
    import scipy.special as sc

    from probabilit_amd import native

    j = np.arange(3841, dtype=np.float64)
    w = np.concatenate([-80.0 + (j[:, None] + np.array([0.0, 0.25, 0.5, 0.75])[None, :]).ravel() / 32.0,
                        np.nextafter(-80.0 + j / 32.0, -np.inf), np.nextafter(-80.0 + j / 32.0, np.inf)])
    p = np.where(w > 0, 1.0 - 1.0 / (1.0 + np.exp(w)), 1.0 / (1.0 + np.exp(-w)))
    p = p[(p > 0) & (p < 1)]
    out = native.ppf("gamma", p, a=a)
    exp = sc.gammaincinv(a, p)
    assert_close(out, exp, rtol=RTOL, what=f"gamma(a={a}) guide intervals")


@pytest.mark.parametrize("mu", [0.3, 4.0, 30.0, 250.0, 2500.0, 20000.0])
def test_poisson_table_every_boundary(gpu, mu):
    """scipy's poisson ppf at every table boundary: for every k with pdtr(k, mu) in (1e-300, 1 - 1e-12),
    q = pdtr(k, mu) exactly, one ulp either side, 40 offsets of 1e-16 .. 1e-6 relative above it
    (where scipy's pdtrik-based answer falls to k - 1 hundreds of times) and 1e-6 either side, plus
    the last quantiles below 1.  The device answers the definition from its CDF table and runs
    scipy's cdflib search (pbh_cdflib.h, bit for bit with scipy.special.pdtrik on the host:
    tests/test_special_host.py) inside the window above each CDF value and in scipy's deep tail, so
    it must equal scipy.stats.poisson.ppf at every q.  The scalar-mu LDS table (mu <= 8900), the
    global table (mu = 2e4) and the per-row (composite) search must agree bit for bit.  The counts go
    to records/."""
    import scipy.special as sc

    from conftest import record
    from oracle.ppf import ppf as ref_ppf
    from probabilit_amd import native

    rng = np.random.default_rng(int(mu))
    k = np.arange(0, int(mu + 40 * np.sqrt(mu) + 40), dtype=np.float64)
    c = sc.pdtr(k, mu)
    c = c[(c > 1e-300) & (c < 1.0 - 1e-12)]
    q = np.concatenate([c, np.nextafter(c, 0.0), np.nextafter(c, 1.0), c * (1.0 - 1e-6), c * (1.0 + 1e-6)] +
                       [c * (1.0 + 10.0 ** rng.uniform(-16, -6, c.size)) for _ in range(40)] +
                       [1.0 - np.arange(1, 64) * 2.0**-53])
    q = q[(q > 0) & (q < 1)]
    out, exp = native.ppf("poisson", q, mu=mu), ref_ppf("poisson", q, mu=mu)
    per_row = native.ppf("poisson", q, mu=np.full(q.shape, mu))
    np.testing.assert_array_equal(per_row, out)
    table = sc.pdtr(np.arange(0, int(mu + 60 * np.sqrt(mu) + 80), dtype=np.float64), mu)
    definition = np.searchsorted(table, q, side="left").astype(np.float64)
    diff = out != exp
    record(f"poisson_boundaries_mu{mu:g}", {
        "mu": mu, "quantiles": int(q.size), "scipy_below_definition": int(np.count_nonzero(exp < definition)),
        "scipy_off_definition": int(np.count_nonzero(exp != definition)), "device_differs_from_scipy": int(diff.sum())})
    np.testing.assert_array_equal(out, exp)


@pytest.mark.parametrize("name,kw,q0", [("norm", dict(loc=2.0, scale=3.0), None), ("norm", dict(loc=-5.0, scale=0.5), None),
                                        ("lognorm", dict(s=0.5, loc=-1.0, scale=1.0), 0.5),
                                        ("lognorm", dict(s=2.0, loc=-3.0, scale=0.7), None)])
def test_norm_lognorm_cancellation_guard(gpu, name, kw, q0):
    """Where loc + scale·z (norm) or loc + scale·exp(s·z) (lognorm) cancels to near zero, a
    1e-15 difference in z becomes ~1e-9 relative in x: there the kernels take Cephes' ndtri, bit
    for bit with scipy, instead of PPND16 (normal_guard, pbh_ppf_core.h).  Quantiles packed around
    the zero crossing, plain and fused-LHS paths, within 1e-10 relative of scipy."""
    import scipy.stats

    from probabilit_amd import native

    dist = getattr(scipy.stats, name)(**kw)
    if q0 is None:
        q0 = float(dist.cdf(0.0))
    offs = np.concatenate([-np.logspace(-15, -3, 400), [0.0], np.logspace(-15, -3, 400)])
    q = np.clip(q0 + offs, 1e-300, 1 - 2.0**-53)
    q = np.concatenate([q, np.nextafter(q0, 0.0) - np.arange(50) * 2.0**-54, np.nextafter(q0, 1.0) + np.arange(50) * 2.0**-53])
    ref = dist.ppf(q)
    got = native.ppf(name, q, **kw)
    # norm: bit for bit there.  lognorm: z is Cephes' bit for bit, but exp(s z) ~ 1 comes from the
    # device's exp, within 1 ulp of libm's, and loc + scale exp(s z) keeps that ulp absolutely
    # (x ~ 1e-15 next to the crossing of lognorm(0.5, loc=-1): one ulp of 1 is 6% of x)
    atol = 0.0 if name == "norm" else 4 * np.spacing(abs(kw["loc"]))
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=atol)
