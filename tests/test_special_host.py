"""CPU sweep of the device special functions (pbh_special.h compiled for the host by
tests/native/special_host.cpp) against scipy 1.15.3, the reference's ppf backend
(modeling.py:807 -> scipy.special.ndtri / gammaincinv / pdtr).

Gate: 1e-10 relative (BASELINE north_star).  The host build uses glibc's libm where the
device uses its own math library, so this pins the algorithms; tests/test_gpu_ppf.py pins
the device results."""

import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest
import scipy.special as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRC = os.path.join(HERE, "native", "special_host.cpp")
OUT = os.path.join(HERE, "native", "_build", "libpbh_special_host.so")


@pytest.fixture(scope="module")
def sfh():
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    if hipcc is None:
        pytest.skip("hipcc not available")
    deps = [SRC] + [os.path.join(ROOT, "probabilit_amd", "csrc", f) for f in ("pbh_special.h", "pbh_special_ext.h", "pbh_common.h",
                                                                            "pbh_tables.inc", "pbh_cdflib.h",
                                                                            "pbh_glibc.h", "pbh_glibc_tables.inc", "pbh_special.h")]
    if not os.path.exists(OUT) or any(os.path.getmtime(d) > os.path.getmtime(OUT) for d in deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        subprocess.run([hipcc, "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
                        "-I", os.path.join(ROOT, "probabilit_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                        SRC, "-o", OUT], check=True, capture_output=True)
    return ctypes.CDLL(OUT)


def _call(lib, fn, *scalars_then_array):
    *scal, arr = scalars_then_array
    arr = np.ascontiguousarray(arr, dtype=np.float64)
    out = np.empty_like(arr)
    P = ctypes.c_void_p
    args = [ctypes.c_double(s) for s in scal]
    getattr(lib, fn)(*args, P(arr.ctypes.data), ctypes.c_long(arr.size), P(out.ctypes.data))
    return out


def _quantiles():
    rng = np.random.default_rng(0)
    return np.concatenate([rng.random(60000), 1 - 10 ** rng.uniform(-16, -1, 20000),
                           10 ** rng.uniform(-300, -1, 20000), 10 ** rng.uniform(-323.5, -300, 2000),
                           [0.0, 5e-324, 1e-300, 2.0 ** -53, 0.5, 1 - 2.0 ** -53, 1.0]])


def _rel(x, ref):
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.abs(x - ref) / np.abs(ref)
    r[(x == ref) | (np.isnan(x) & np.isnan(ref))] = 0.0
    return r


def test_ndtri_matches_scipy(sfh):
    q = _quantiles()
    r = _rel(_call(sfh, "sfh_ndtri", q), sp.ndtri(q))
    assert r.max() <= 1e-13


def test_ppnd16_matches_scipy(sfh):
    """sf::ppnd16 (AS 241, the device norm / lognorm ppf and van der Waerden scores) against scipy's
    ndtri: within 2e-15 relative everywhere (quantiles from 1e-300 to 1 - 1e-16, the van der
    Waerden grid), about one ulp on average; infinities at 0 and 1, NaN outside."""
    rng = np.random.default_rng(5)
    q = np.concatenate([_quantiles(), rng.random(1_000_000), 10.0 ** (-rng.random(200_000) * 300),
                        1.0 - 10.0 ** (-rng.random(200_000) * 16), np.arange(1, 200_002) / 200_002.0,
                        [0.0, 1.0, -0.5, 1.5, np.nan, 0.075, 0.925, 0.5, np.nextafter(0.075, 1)]])
    got = _call(sfh, "sfh_ppnd16", q)
    ref = sp.ndtri(q)
    assert (np.isnan(got) == np.isnan(ref)).all()
    r = _rel(got, ref)
    assert r.max() <= 2e-15, r.max()
    fin = np.isfinite(ref) & (ref != 0.0)
    assert np.mean(np.abs(got[fin] - ref[fin]) / np.spacing(np.abs(ref[fin]))) < 1.5


@pytest.mark.parametrize("a", [0.05, 0.1, 0.3, 0.7, 1.0, 2.0, 5.0, 20.0, 45.0, 100.0, 250.0, 1e3, 1e4, 1e5])
def test_gammaincinv_and_guided_table(sfh, a):
    q = _quantiles()
    ref = sp.gammaincinv(a, q)
    direct = _call(sfh, "sfh_igami", a, q)
    guided = _call(sfh, "sfh_igami_guided", a, q)
    assert (np.isnan(direct) == np.isnan(ref)).all() and (np.isnan(guided) == np.isnan(ref)).all()
    assert _rel(direct, ref).max() <= 1e-12, "igami restatement"
    assert _rel(guided, ref).max() <= 1e-10, "guide-table igami"


@pytest.mark.parametrize("mu", [0.5, 4.0, 30.0, 1000.0])
def test_pdtr_matches_scipy(sfh, mu):
    k = np.arange(0, int(mu + 20 * np.sqrt(mu) + 40), dtype=np.float64)
    r = _rel(_pdtr(sfh, k, mu), sp.pdtr(k, mu))
    assert r.max() <= 1e-12


def _pdtr(lib, k, mu):
    k = np.ascontiguousarray(k)
    out = np.empty_like(k)
    P = ctypes.c_void_p
    lib.sfh_pdtr(P(k.ctypes.data), ctypes.c_double(mu), ctypes.c_long(k.size), P(out.ctypes.data))
    return out


@pytest.mark.parametrize("a,floor", [(0.05, 0.6), (0.1, 0.85), (0.3, 0.999), (0.7, 0.999), (2.0, 0.999), (45.0, 0.999),
                                     (1e4, 0.999)])
def test_guide_table_mostly_interpolates(sfh, a, floor):
    """The quintic guide must cover (nearly) the whole grid; otherwise the Halley fallback
    silently carries the cost.  For small a the lower grid maps to x below 1e-290 (x ~ p^(1/a)),
    which is deliberately left to igami: on the log-odds grid (w from -80) that is w < -33 for
    a = 0.05 (p < ~1e-14.5), 39% of the grid, and w < -60 for a = 0.1."""
    sfh.sfh_guide_ok_fraction.restype = ctypes.c_double
    assert sfh.sfh_guide_ok_fraction(ctypes.c_double(a)) >= floor


# ---------------------------------------------------------------- extended distributions
def _arr(lib, fn, *scal, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    out = np.empty_like(x)
    f = getattr(lib, fn)
    f.restype = None
    cargs = [ctypes.c_double(v) for v in scal]
    f(*cargs, x.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(x.size), out.ctypes.data_as(ctypes.c_void_p))
    return out


def _rel(a, e):
    with np.errstate(all="ignore"):
        return np.nanmax(np.abs(a - e) / np.maximum(np.abs(e), 1e-300))


def test_log_ndtr_and_ndtri_exp(sfh):
    x = np.concatenate([-np.logspace(-3, 2.5, 400), np.linspace(-5, 8, 400)])
    assert _rel(_arr(sfh, "sfh_log_ndtr", x=x), sp.log_ndtr(x)) < 1e-13
    y = np.concatenate([-np.logspace(-12, 4, 500), [-1e-300, -0.1454134578688591, -2.0, -2.0000001]])
    assert _rel(_arr(sfh, "sfh_ndtri_exp", x=y), sp.ndtri_exp(y)) < 1e-13


@pytest.mark.parametrize("a,b", [(-1.0, 1.0), (3.0, 3.3), (-3.3, -3.0), (-0.5, 2.0), (0.1, 8.0), (-40, -39.5)])
def test_truncnorm_ppf(sfh, a, b):
    import scipy.stats as st

    q = np.concatenate([np.linspace(1e-6, 1 - 1e-6, 999), [1e-300, 0.5, 1 - 2**-53]])
    got = _arr(sfh, "sfh_truncnorm_ppf", a, b, x=q)
    ref = st.truncnorm(a, b).ppf(q)
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-13)


@pytest.mark.parametrize("a,b", [(0.5, 0.5), (2.0, 3.0), (3.4, 2.6), (7.0, 5.0), (0.1, 10.0), (50.0, 80.0),
                                 (1.0, 1.0), (200.0, 0.7)])
def test_incbet_and_beta_ppf(sfh, a, b):
    x = np.linspace(0, 1, 1001)
    np.testing.assert_allclose(_arr(sfh, "sfh_incbet", a, b, x=x), sp.betainc(a, b, x), rtol=1e-12, atol=1e-300)
    # q >= 2^-53 / n covers every generator here; Boost (scipy) gives NaN for some q ~ 1e-300
    # where the root underflows its internal scaling, which no generated quantile reaches
    q = np.concatenate([np.linspace(1e-9, 1 - 1e-9, 2001), [1e-30, 2.0**-53 / 1e8, 0.5, 1 - 2**-52]])
    got = _arr(sfh, "sfh_beta_ppf", a, b, x=q)
    np.testing.assert_allclose(got, sp.betaincinv(a, b, q), rtol=1e-10, atol=1e-300)


@pytest.mark.parametrize("a,b", [(3.4, 2.6), (7.0, 5.0), (2.0, 3.0), (1.0, 1.0), (0.5, 0.5), (0.1, 10.0),
                                 (50.0, 80.0), (200.0, 0.7), (1.3, 4.7)])
def test_beta_guide(sfh, a, b):
    """The beta guide table (sfx::beta_ppf_guided: quintic Hermite of logit x in logit q, checked
    at every interval's midpoint) against scipy's betaincinv, and its coverage of the grid."""
    rng = np.random.default_rng(int(a * 10 + b))
    q = np.concatenate([rng.random(200_000), np.linspace(1e-9, 1 - 1e-9, 2001),
                        [1e-30, 2.0**-53 / 1e8, 0.5, 1 - 2**-52]])
    x = np.ascontiguousarray(q)
    out = np.empty(q.size + 1)
    f = sfh.sfh_beta_guided
    f.restype = None
    f(ctypes.c_double(a), ctypes.c_double(b), x.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(q.size),
      out.ctypes.data_as(ctypes.c_void_p))
    got, coverage = out[:-1], out[-1]
    np.testing.assert_allclose(got, sp.betaincinv(a, b, q), rtol=1e-10, atol=1e-300)
    # the measured share of guide intervals that pass the midpoint check: all of them for these
    # shapes except (0.1, 10), 99.84% (a regression that sent draws to the slow betaincinv path
    # would show here)
    assert coverage >= (0.998 if min(a, b) < 0.2 else 1.0), coverage


@pytest.mark.parametrize("n,p", [(1, 0.3), (10, 0.5), (37, 0.01), (1000, 0.7), (20, 0.0), (20, 1.0)])
def test_binom_ppf(sfh, n, p):
    import scipy.stats as st

    q = np.random.default_rng(n).random(5000)
    got = _arr(sfh, "sfh_binom_ppf", n, p, x=q)
    np.testing.assert_array_equal(got, st.binom(n, p).ppf(q))


def test_log_tab_is_correctly_rounded(sfh):
    """sf::log_tab (the table-driven log of ndtri's tail and the gamma log-odds) against a
    60-digit log: the result is the correctly rounded value, or a neighbour only where the
    exact value lies within ~0.01 ulp of a rounding midpoint."""
    import mpmath

    mpmath.mp.dps = 40
    rng = np.random.default_rng(5)
    x = np.concatenate([10 ** rng.uniform(-300, 300, 4000), rng.uniform(0.5, 2.0, 4000),
                        1.0 + rng.uniform(-2.0 ** -7, 2.0 ** -7, 2000), 10 ** rng.uniform(-17, -0.8, 4000),
                        rng.uniform(2.0, 40.0, 4000), [1.0, 2.0, 0.5, 0.6875, 1.375, 1.0078125, 2.0 ** -1022,
                                                       1.7976931348623157e308, 1 + 2.0 ** -52, 1 - 2.0 ** -53]])
    got = _call(sfh, "sfh_log_tab", x)
    worst = 0.0
    for xi, gi in zip(x, got):
        ex = mpmath.log(mpmath.mpf(float(xi)))
        ulp = np.spacing(abs(float(ex))) if float(ex) != 0.0 else 5e-324
        err = abs(float((mpmath.mpf(float(gi)) - ex) / ulp)) if float(ex) != 0.0 else abs(gi)
        worst = max(worst, err)
    assert worst < 0.52, worst
    for special in (0.0, -1.0, np.inf, np.nan, 5e-324, 1e-310):
        a = _call(sfh, "sfh_log_tab", np.array([special]))[0]
        with np.errstate(divide="ignore", invalid="ignore"):
            b = np.log(special)
        assert (np.isnan(a) and np.isnan(b)) or a == b, (special, a, b)


@pytest.mark.parametrize("lo,hi", [(1e-17, 0.1353352832366127), (2.0, 40.0), (1e-8, 1e8), (1e-300, 1e300)])
def test_log_tab_agrees_with_libm(sfh, lo, hi):
    """Against glibc's log on 2e6 points of each range ndtri's tail and the gamma log-odds
    use: never more than 1 ulp apart, and equal on all but ~1e-4 of them (where they differ,
    log_tab is the correctly rounded one in 162 of 163 sampled cases: glibc's own bound is
    0.52 ulp)."""
    counts = np.zeros(2, dtype=np.int64)
    n = 2_000_000
    sfh.sfh_log_tab_vs_libm(ctypes.c_double(lo), ctypes.c_double(hi), ctypes.c_long(n), ctypes.c_ulonglong(7),
                            ctypes.c_void_p(counts.ctypes.data))
    assert counts[1] == 0, counts
    assert counts[0] <= n * 2e-4, counts


def test_exp_tab_is_correctly_rounded(sfh):
    """sf::exp_tab (the gamma guide's e^y) against a 40-digit exp on [-700, 700]."""
    import mpmath

    mpmath.mp.dps = 40
    rng = np.random.default_rng(6)
    y = np.concatenate([rng.uniform(-700, 700, 8000), rng.uniform(-3, 3, 4000), rng.uniform(-1e-3, 1e-3, 1000),
                        [0.0, 1.0, -1.0, 700.0, -700.0, 0.5 * np.log(2), np.log(2), 1e-300]])
    got = _call(sfh, "sfh_exp_tab", y)
    worst = 0.0
    for yi, gi in zip(y, got):
        ex = mpmath.exp(mpmath.mpf(float(yi)))
        worst = max(worst, abs(float((mpmath.mpf(float(gi)) - ex) / np.spacing(float(ex)))))
    assert worst < 0.52, worst


@pytest.mark.parametrize("lo,hi", [(-700.0, 700.0), (-40.0, 5.0)])
def test_exp_tab_agrees_with_libm(sfh, lo, hi):
    """Never more than 1 ulp from glibc's exp; equal on all but ~1e-3 of the points (both are
    within 0.52 ulp; where they differ each is the better rounded one about half the time).  Its
    one use, the gamma guide's interpolated log x, is itself accurate to ~1e-12."""
    counts = np.zeros(2, dtype=np.int64)
    n = 2_000_000
    sfh.sfh_exp_tab_vs_libm(ctypes.c_double(lo), ctypes.c_double(hi), ctypes.c_long(n), ctypes.c_ulonglong(9),
                            ctypes.c_void_p(counts.ctypes.data))
    assert counts[1] == 0, counts
    assert counts[0] <= n * 3e-3, counts


# ---------------------------------------------------------------- poisson ppf: cdflib's pdtrik
# scipy's poisson._ppf is ceil(pdtrik(q, mu)) with a one-step pdtr correction downwards
# (modeling.py:807 -> scipy/stats/_discrete_distns.py); pdtrik is cdflib's cdfpoi (dinvr + dzror
# over gratio).  pbh_cdflib.h restates it; the device answers the definition from its CDF table
# and runs the restatement for the lanes in the window above each CDF value where the two can
# differ.  These tests pin the restatement against scipy.special.pdtrik / scipy.stats.poisson.


def test_cdflib_helpers_match_their_functions(sfh):
    """gratio's helpers with their published constants: Morris' Gamma on [1, 20), erfc1 (erfc and
    exp(x^2) erfc) and rlog (x - 1 - ln x), against scipy / a 30-digit reference."""
    import mpmath

    mpmath.mp.dps = 30
    a = np.linspace(1.0, 19.99, 800)
    np.testing.assert_allclose(_call(sfh, "sfh_cdflib_gamma", a), sp.gamma(a), rtol=1e-14)
    x = np.linspace(-5.0, 26.0, 4000)
    np.testing.assert_allclose(_call(sfh, "sfh_erfc1", 0, x), sp.erfc(x), rtol=5e-15)
    np.testing.assert_allclose(_call(sfh, "sfh_erfc1", 1, x), sp.erfcx(x), rtol=5e-15)
    x = np.linspace(0.3, 3.0, 1500)
    ref = np.array([float(mpmath.mpf(float(v)) - 1 - mpmath.log(float(v))) for v in x])
    np.testing.assert_allclose(_call(sfh, "sfh_rlog", x), ref, rtol=5e-15, atol=1e-300)


@pytest.mark.parametrize("a", [1.0, 2.5, 3.0, 5.3, 12.0, 17.5, 21.0, 30.2, 100.0, 274.1])
def test_gratio_matches_incomplete_gamma(sfh, a):
    """gratio's P and Q (series, continued fraction, finite sums, asymptotic and Temme branches)
    within its design accuracy of scipy's gammainc / gammaincc."""
    x = a * np.concatenate([np.linspace(0.05, 3.0, 400), 1.0 + np.linspace(-1e-3, 1e-3, 60)])
    p, q = _call(sfh, "sfh_gratio_p", a, x), _call(sfh, "sfh_gratio_q", a, x)
    np.testing.assert_allclose(p, sp.gammainc(a, x), rtol=5e-13, atol=1e-300)
    np.testing.assert_allclose(q, sp.gammaincc(a, x), rtol=5e-13, atol=1e-300)


def test_glibc_exp_log_bit_exact(sfh):
    """pbh_glibc.h (glibc 2.35's table-driven exp and log with the FMA build's fused multiply-adds,
    the libm scipy's cdflib calls) against this image's libm, bit for bit, over the ranges gratio and
    its helpers reach, the tails, subnormals and special values."""
    import ctypes.util

    libm = ctypes.CDLL(ctypes.util.find_library("m"))
    libm.exp.restype = libm.log.restype = ctypes.c_double
    libm.exp.argtypes = libm.log.argtypes = [ctypes.c_double]
    rng = np.random.default_rng(1)
    xe = np.concatenate([rng.uniform(-745.2, 709.8, 200000), rng.uniform(-1, 1, 100000), rng.normal(0, 30, 100000),
                         10.0 ** rng.uniform(-20, -1, 20000), [0.0, -0.0, 1e-300, -746.0, 710.0, np.inf, -np.inf,
                                                                  -708.4, -744.5, 512.0, -512.0, 1023.9]])
    xl = np.concatenate([10.0 ** rng.uniform(-320, 308, 200000), rng.uniform(0.9, 1.1, 100000),
                         rng.uniform(0.5, 2.0, 100000), [1.0, np.nextafter(1.0, 2), np.nextafter(1.0, 0), 5e-324,
                                                         2.2250738585072014e-308, np.inf, 0.0]])
    want_e = np.array([libm.exp(float(v)) for v in xe])
    want_l = np.array([libm.log(float(v)) for v in xl])
    np.testing.assert_array_equal(_call(sfh, "sfh_glibc_exp", xe), want_e)
    np.testing.assert_array_equal(_call(sfh, "sfh_glibc_log", xl), want_l)
    # pow on the arguments the Cephes incomplete gamma gives it (igam_fac: (x / fac)^a, a < 200)
    # and beyond
    libm.pow.restype = ctypes.c_double
    libm.pow.argtypes = [ctypes.c_double, ctypes.c_double]
    px = np.concatenate([rng.uniform(0.5, 1.5, 100000), 10.0 ** rng.uniform(-300, 300, 50000)])
    py = np.concatenate([rng.uniform(0.5, 200.0, 100000), rng.uniform(-1.0, 1.0, 50000)])
    got = np.empty_like(px)
    P = ctypes.c_void_p
    sfh.sfh_glibc_pow(P(px.ctypes.data), P(py.ctypes.data), ctypes.c_long(px.size), P(got.ctypes.data))
    np.testing.assert_array_equal(got, np.array([libm.pow(float(a), float(b)) for a, b in zip(px, py)]))


@pytest.mark.parametrize("mu", [1e-3, 0.5, 1.0, 2.0, 3.0, 4.0, 17.3, 30.0, 250.0, 2500.0, 1e5])
def test_pdtrik_matches_scipy(sfh, mu):
    """The restated cdfpoi search against scipy.special.pdtrik on uniform p and both tails: bit for
    bit.  (scipy 1.15.3's C cdflib carries alog10, rt2pin, rtpi, 1/3 and Gamma's Stirling constant
    to full precision, runs the finite sums as t *= x / c, sums all 20 stored series terms, tests
    the series tail before its first term, and forms erfc1's large-x ratio before the multiply by
    1/x^2: each read from its compiled code; exp / log are glibc's, pbh_glibc.h.)"""
    rng = np.random.default_rng(int(mu * 1000))
    p = np.concatenate([rng.random(20000), 10.0 ** rng.uniform(-300, 0, 3000), 1 - 10.0 ** rng.uniform(-16, -1, 3000)])
    got, ref = _call(sfh, "sfh_pdtrik", mu, p), sp.pdtrik(p, mu)
    np.testing.assert_array_equal(got, ref)


def test_pdtrik_windows_random_means(sfh):
    """pdtrik bit for bit on p packed next to every CDF value (the windows where its root search
    decides the integer) for 60 log-uniform means from 0.02 to 3e4."""
    rng = np.random.default_rng(11)
    for mu in np.exp(rng.uniform(np.log(0.02), np.log(3e4), 60)):
        k = np.arange(0, int(mu + 12 * np.sqrt(mu) + 20), dtype=float)
        c = sp.pdtr(k, mu)
        c = c[(c > 0) & (c < 1)]
        p = np.concatenate([c * (1 + 10.0 ** rng.uniform(-16, -6, c.size)), np.nextafter(c, 2), rng.random(300)])
        p = p[(p > 0) & (p < 1)]
        np.testing.assert_array_equal(_call(sfh, "sfh_pdtrik", float(mu), p), sp.pdtrik(p, mu), err_msg=str(mu))


def _window_quantiles(mu, per=200, seed=3):
    """q just above every CDF value pdtr(k, mu) in (0, 1) (offsets 1e-18 .. 1e-4 relative, the
    value itself and the next double), plus uniform q."""
    rng = np.random.default_rng(seed)
    k = np.arange(0, int(mu + 14 * np.sqrt(mu) + 25), dtype=np.float64)
    c = sp.pdtr(k, mu)
    c = c[(c > 0) & (c < 1)]
    q = np.concatenate([ci * (1 + 10.0 ** rng.uniform(-18, -4, per)) for ci in c] + [np.nextafter(c, 2), c,
                                                                                    rng.random(20000)])
    return q[(q > 0) & (q < 1)], c


@pytest.mark.parametrize("mu", [0.3, 4.0, 30.0, 100.0, 2500.0])
def test_poisson_ppf_windows_equal_scipy(sfh, mu):
    """The device's poisson ppf (definition from the CDF table, scipy's pdtrik search inside the
    window above each CDF value) against scipy.stats.poisson.ppf on q packed into those windows
    (where the definition alone differs from scipy hundreds of times) and on uniform q: equal at
    every q, no allowance."""
    import scipy.stats as st

    q, c = _window_quantiles(mu)
    ref = st.poisson(mu).ppf(q)
    got = _call(sfh, "sfh_poisson_ppf_device", mu, q)
    np.testing.assert_array_equal(got, ref)


def test_poisson_ppf_random_means_exact(sfh):
    """The device's poisson ppf rule (definition, scipy's search inside the windows and below
    kPoissonDeepTail) equals scipy.stats.poisson.ppf for 40 log-uniform means from 0.05 to 1e5 on q
    packed next to every CDF value, on log-uniform q down to 1e-300, and on uniform q."""
    import scipy.stats as st

    rng = np.random.default_rng(21)
    for mu in np.exp(rng.uniform(np.log(0.05), np.log(1e5), 40)):
        q, _ = _window_quantiles(float(mu), per=8, seed=int(mu * 7) % 1000)
        q = np.concatenate([q[:-20000], 10.0 ** rng.uniform(-300, -1, 3000), rng.random(3000)])
        kdef = _smallest_k(q, float(mu))
        out = np.empty_like(q)
        sfh.sfh_poisson_rule(ctypes.c_double(mu), q.ctypes.data_as(ctypes.c_void_p),
                             kdef.ctypes.data_as(ctypes.c_void_p), ctypes.c_long(q.size),
                             out.ctypes.data_as(ctypes.c_void_p))
        np.testing.assert_array_equal(out, st.poisson(mu).ppf(q), err_msg=str(mu))


def _smallest_k(q, mu):
    """the definition: smallest k with pdtr(k, mu) >= q (scipy's pdtr, vectorised)"""
    table = sp.pdtr(np.arange(0, int(mu + 40 * np.sqrt(mu) + 60), dtype=np.float64), mu)
    return np.searchsorted(table, q, side="left").astype(np.float64)


def test_poisson_window_covers_scipy_deviations(sfh):
    """Every q where scipy's answer is below the definition lies inside the device's window
    (win[k] = Q(k + delta, mu) (1 + 2^-40), delta = 1.25e-10 (k - 1): dzror's relative tolerance
    with 25% to spare), over q packed into the windows of every CDF value."""
    import scipy.stats as st

    for mu in (0.3, 1.0, 4.0, 12.0, 30.0, 100.0, 250.0, 1000.0):
        q, c = _window_quantiles(mu, per=300, seed=7)
        ref = st.poisson(mu).ppf(q)
        k = _smallest_k(q, mu)
        dev = (ref != k) & (q >= 1e-150)  # below: cdflib's gratio underflows (scipy's deep tail)
        assert np.all(ref[dev] == k[dev] - 1), mu
        hi = _call(sfh, "sfh_poisson_window_hi", mu, k[dev])
        assert np.all(q[dev] < hi), (mu, q[dev][q[dev] >= hi][:4])


# ---- round 5 distributions on the host (pbh_special_ext.h), against scipy
@pytest.mark.parametrize("p", [0.3, 0.01, 0.999, 1.0, 1e-6])
def test_geom_ppf(sfh, p):
    import scipy.stats as st

    q = _quantiles()
    q = q[(q > 0) & (q < 1)]
    with np.errstate(divide="ignore"):
        ref = st.geom(p).ppf(q)
    np.testing.assert_array_equal(_call(sfh, "sfh_geom_ppf", p, q), ref)


@pytest.mark.parametrize("low,high", [(2, 7), (-5, 100), (0, 1), (-1e6, 3e6)])
def test_randint_ppf(sfh, low, high):
    import scipy.stats as st

    q = _quantiles()
    q = q[(q > 0) & (q < 1)]
    np.testing.assert_array_equal(_call(sfh, "sfh_randint_ppf", low, high, q), st.randint(low, high).ppf(q))


@pytest.mark.parametrize("n,p", [(3.5, 0.4), (1, 0.5), (20, 0.9), (0.5, 0.05), (100, 0.3)])
def test_nbinom_ppf(sfh, n, p):
    import scipy.stats as st

    q = np.random.default_rng(int(n * 10)).random(20000)
    np.testing.assert_array_equal(_call(sfh, "sfh_nbinom_ppf", n, p, q), st.nbinom(n, p).ppf(q))


@pytest.mark.parametrize("df", [0.5, 1.0, 2.5, 5.0, 30.0, 300.0, 1e4, 9e4, 1e5, 3e7, np.inf])
def test_t_ppf(sfh, df):
    import scipy.stats as st

    rng = np.random.default_rng(3)
    q = np.concatenate([rng.random(20000), 10.0 ** rng.uniform(-15, -1, 2000), 1 - 10.0 ** rng.uniform(-15, -1, 2000)])
    np.testing.assert_allclose(_call(sfh, "sfh_t_ppf", df, q), st.t(df).ppf(q), rtol=1e-10)


@pytest.mark.parametrize("a", [0.1, 1.0, 2.5, 30.0, 500.0])
def test_invgamma_ppf(sfh, a):
    import scipy.stats as st

    q = _quantiles()
    q = q[(q > 0) & (q < 1)]
    np.testing.assert_allclose(_call(sfh, "sfh_invgamma_ppf", a, q), st.invgamma(a).ppf(q), rtol=1e-12)
