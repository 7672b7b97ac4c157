"""Distributions beyond the base set on the GPU (beta / PERT, truncnorm,
binom, bernoulli and the distributions.py constructors) against scipy's ppf on the same
quantiles (the reference's computation, modeling.py:807) and against outputs of the reference
itself (tests/golden/dists.npz).  Gate: 1e-10 relative for floating point, exact for discrete."""

import numpy as np
import pytest

from conftest import assert_close, golden

pytestmark = pytest.mark.gpu


def _q(n, seed):
    q = np.random.default_rng(seed).random(n)
    return np.concatenate([q, [0.0, 2.0**-53 / 1e8, 1e-12, 0.5, 1 - 1e-12, 1 - 2.0**-53, 1.0]])


@pytest.mark.parametrize("kw", [dict(a=0.5, b=0.5), dict(a=3.4, b=2.6, loc=0, scale=10), dict(a=7.0, b=5.0),
                                dict(a=0.1, b=10.0), dict(a=50.0, b=80.0, loc=-1.0, scale=3.0), dict(a=1.0, b=1.0)])
def test_beta_ppf(gpu, kw):
    import scipy.stats

    from probabilit_amd import native

    q = _q(20_000, 1)
    assert_close(native.ppf("beta", q, **kw), scipy.stats.beta(**kw).ppf(q), rtol=1e-10, atol=1e-300, what=f"{kw}")


@pytest.mark.parametrize("kw", [dict(a=3.0, b=3.3), dict(a=-1.0, b=1.0, loc=2.0, scale=0.5), dict(a=-3.3, b=-3.0),
                                dict(a=-0.5, b=2.0), dict(a=0.1, b=8.0), dict(a=-40.0, b=-39.5)])
def test_truncnorm_ppf(gpu, kw):
    import scipy.stats

    from probabilit_amd import native

    q = _q(20_000, 2)
    ref = scipy.stats.truncnorm(**kw).ppf(q)
    assert_close(native.ppf("truncnorm", q, **kw), ref, rtol=1e-10, atol=1e-13, what=f"{kw}")


@pytest.mark.parametrize("name,kw", [("binom", dict(n=1, p=0.3)), ("binom", dict(n=20, p=0.3)),
                                     ("binom", dict(n=1000, p=0.7, loc=2)), ("binom", dict(n=37, p=0.01)),
                                     ("binom", dict(n=5, p=0.0)), ("binom", dict(n=5, p=1.0)),
                                     ("binom", dict(n=2.5, p=0.5)), ("bernoulli", dict(p=0.25)),
                                     ("bernoulli", dict(p=0.0))])
def test_discrete_ppf_exact(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native

    q = _q(50_000, 3)
    np.testing.assert_array_equal(native.ppf(name, q, **kw), getattr(scipy.stats, name)(**kw).ppf(q))


def test_composite_beta_parameters(gpu):
    import scipy.stats

    from probabilit_amd import native

    n = 10_000
    rng = np.random.default_rng(4)
    q, a, b = rng.random(n), 1 + 3 * rng.random(n), 0.5 + rng.random(n)
    assert_close(native.ppf("beta", q, a=a, b=b), scipy.stats.beta(a=a, b=b).ppf(q), rtol=1e-10, atol=1e-300)


def test_distribution_constructors_vs_reference(gpu):
    """distributions.py constructors sampled with method=None: the reference's own outputs."""
    from probabilit_amd import distributions as dists
    from probabilit_amd.modeling import Distribution as D

    z = golden("dists.npz")
    assert_close(dists.PERT(0, 6, 10).sample(2000, random_state=0), z["pert"], what="PERT")
    assert_close(dists.TruncatedNormal(loc=0, scale=1, low=3, high=3.3).sample(2000, random_state=0), z["tnorm"],
                 what="TruncatedNormal")
    assert_close(dists.Lognormal(mean=2, std=1).sample(999, random_state=0), z["lognorm_ms"], what="Lognormal")
    assert_close(dists.Lognormal(mean=D("expon", scale=1), std=1).sample(500, random_state=0), z["lognorm_comp"],
                 what="Lognormal composite")
    assert_close(dists.Triangular(low=1, mode=5, high=9).sample(1000, random_state=3), z["tri"], what="Triangular")
    np.testing.assert_array_equal(D("binom", n=20, p=0.3).sample(3000, random_state=2), z["binom"])
    np.testing.assert_array_equal(D("bernoulli", p=0.25).sample(3000, random_state=2), z["bern"])
    assert_close(D("beta", 0.5, 0.5).sample(2000, random_state=5), z["beta_small"], what="beta(0.5, 0.5)")
    assert_close(D("beta", a=D("uniform", loc=1, scale=3), b=2.0).sample(1500, random_state=7), z["composite"],
                 what="composite beta")


def test_distributions_docstring_pins(gpu):
    """distributions.py:22-24, 40-55, 70-74, 84-88, 105-111."""
    from probabilit_amd import distributions as dists
    from probabilit_amd.modeling import Distribution as D

    np.testing.assert_array_equal(dists.TruncatedNormal(loc=0, scale=1, low=3, high=3.3).sample(7, random_state=0)
                                  .round(3), [3.13, 3.182, 3.146, 3.129, 3.095, 3.159, 3.099])
    s = dists.Lognormal(mean=2, std=1).sample(999, random_state=0)
    assert str(float(np.mean(s))).startswith("2.00173") and str(float(np.std(s))).startswith("1.02675")
    np.testing.assert_allclose(dists.Lognormal(mean=D("expon", scale=1), std=1).sample(5, random_state=0),
                               [0.86196529, 0.69165866, 0.41782557, 1.23340656, 2.90778578], rtol=0, atol=5e-9)
    np.testing.assert_allclose(dists.Lognormal.from_log_params(mu=D("norm"), sigma=1).sample(5, random_state=0),
                               [1.99625633, 1.45244764, 1.19926216, 2.94150961, 4.47459182], rtol=0, atol=5e-9)
    assert repr(dists.PERT(0, 6, 10)) == 'Distribution("beta", a=3.4, b=2.6, loc=0, scale=10)'
    assert repr(dists.PERT(0, 6, 10, gamma=10)) == 'Distribution("beta", a=7.0, b=5.0, loc=0, scale=10)'
    assert repr(dists.Triangular(low=1, mode=5, high=9, low_perc=0, high_perc=1)) == \
        'Distribution("triang", loc=1, scale=8, c=0.5)'


# scipy's closed-form ppf bodies (PBH_DIST_WEIBULL_MIN..CHI2, pbh_ppf_ext.hip closed_ppf01): shapes,
# loc / scale, invalid arguments (NaN, as rv_continuous.ppf) and the support ends at q = 0 / 1
_CLOSED = [("weibull_min", dict(c=1.7)), ("weibull_min", dict(c=0.4, loc=-2.0, scale=3.0)),
           ("weibull_max", dict(c=2.5)), ("weibull_max", dict(c=0.7, loc=1.0, scale=0.5)),
           ("logistic", dict()), ("logistic", dict(loc=3.0, scale=0.2)), ("cauchy", dict()),
           ("cauchy", dict(loc=-1.0, scale=4.0)), ("laplace", dict()), ("laplace", dict(loc=5.0, scale=2.0)),
           ("gumbel_r", dict()), ("gumbel_r", dict(loc=1.0, scale=3.0)), ("gumbel_l", dict(scale=0.5)),
           ("pareto", dict(b=2.62)), ("pareto", dict(b=0.5, loc=-1.0, scale=2.0)), ("loguniform", dict(a=0.01, b=1.0)),
           ("loguniform", dict(a=2.0, b=1e6, loc=1.0, scale=3.0)), ("reciprocal", dict(a=1.0, b=10.0)),
           ("rayleigh", dict()), ("rayleigh", dict(loc=2.0, scale=5.0)), ("lomax", dict(c=1.88)),
           ("lomax", dict(c=0.3, scale=2.0)), ("genextreme", dict(c=-0.1)), ("genextreme", dict(c=0.5)),
           ("genextreme", dict(c=0.0, loc=1.0)), ("gompertz", dict(c=0.95)), ("gompertz", dict(c=4.0, scale=0.1)),
           ("chi2", dict(df=1.0)), ("chi2", dict(df=5.5, loc=1.0, scale=2.0)), ("chi2", dict(df=55.0)),
           ("weibull_min", dict(c=-1.0)), ("pareto", dict(b=0.0)), ("loguniform", dict(a=2.0, b=1.0)),
           ("genextreme", dict(c=np.inf)), ("logistic", dict(scale=-1.0)), ("chi2", dict(df=-2.0))]
# round 4: 30 more closed forms (pbh_ppf_ext.hip closed_ppf01, PBH_DIST_HALFCAUCHY..TRAPEZOID)
_CLOSED2 = [("halfcauchy", dict()), ("halfcauchy", dict(loc=1.0, scale=2.0)), ("halflogistic", dict()),
            ("halfnorm", dict()), ("halfnorm", dict(loc=-1.0, scale=0.5)), ("arcsine", dict()),
            ("hypsecant", dict()), ("powerlaw", dict(a=1.66)), ("powerlaw", dict(a=0.3, scale=4.0)),
            ("genpareto", dict(c=0.1)), ("genpareto", dict(c=-0.5)), ("genpareto", dict(c=0.0)),
            ("fisk", dict(c=3.09)), ("burr", dict(c=10.5, d=4.3)), ("burr", dict(c=0.8, d=0.6, loc=1.0)),
            ("burr12", dict(c=10.0, d=4.0)), ("burr12", dict(c=0.7, d=2.5)), ("exponweib", dict(a=2.89, c=1.95)),
            ("exponpow", dict(b=2.7)), ("bradford", dict(c=0.3)), ("bradford", dict(c=40.0)), ("anglit", dict()),
            ("levy", dict()), ("levy", dict(loc=2.0, scale=0.1)), ("levy_l", dict()), ("gibrat", dict()),
            ("invweibull", dict(c=10.6)), ("invweibull", dict(c=0.7)), ("loglaplace", dict(c=3.25)),
            ("truncexpon", dict(b=4.69)), ("truncexpon", dict(b=0.01)), ("chi", dict(df=0.78)),
            ("chi", dict(df=7.0, scale=2.0)), ("maxwell", dict()), ("nakagami", dict(nu=4.97)),
            ("nakagami", dict(nu=0.6)), ("dweibull", dict(c=2.07)), ("kappa3", dict(a=1.0)),
            ("kappa3", dict(a=0.3)), ("genhalflogistic", dict(c=0.77)), ("alpha", dict(a=3.57)),
            ("fatiguelife", dict(c=29.0)), ("fatiguelife", dict(c=0.3)), ("genlogistic", dict(c=0.41)),
            ("genlogistic", dict(c=5.0)), ("trapezoid", dict(c=0.2, d=0.8)), ("trapezoid", dict(c=0.0, d=1.0)),
            ("trapezoid", dict(c=0.5, d=0.5)), ("trapezoid", dict(c=0.7, d=0.3)), ("genpareto", dict(c=np.nan)),
            ("burr", dict(c=-1.0, d=1.0)), ("powerlaw", dict(a=0.0)), ("erlang", dict(a=3)),
            ("erlang", dict(a=1, loc=1.0, scale=2.0))]


@pytest.mark.parametrize("name,kw", _CLOSED + _CLOSED2)
def test_closed_form_ppf(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native

    q = np.concatenate([_q(20_000, 5), np.linspace(0.29, 0.66, 2001), [-0.5, 1.5, np.nan]])
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    assert_close(native.ppf(name, q, **kw), ref, rtol=1e-10, atol=1e-13, what=f"{name} {kw}")


def test_closed_form_composite_and_sample(gpu):
    """Per-row shapes and loc (composite parameters, modeling.py:796-802) and Node.sample with
    method=None: the reference's RandomState(seed).random((size, 1)) through scipy's ppf."""
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D

    n = 10_000
    rng = np.random.default_rng(6)
    q, c, loc = rng.random(n), 0.2 + 3 * rng.random(n), rng.normal(size=n)
    for name in ("weibull_min", "lomax", "genextreme", "gompertz", "chi2"):
        kw = dict(df=c) if name == "chi2" else dict(c=c)
        assert_close(native.ppf(name, q, loc=loc, **kw), getattr(scipy.stats, name)(loc=loc, **kw).ppf(q),
                     rtol=1e-10, atol=1e-13, what=f"composite {name}")
    a = 0.5 + rng.random(n)
    assert_close(native.ppf("loguniform", q, a=a, b=a * 7.0), scipy.stats.loguniform(a, a * 7.0).ppf(q),
                 what="composite loguniform")
    for name, kw in [("weibull_min", dict(c=1.5)), ("gumbel_r", dict(loc=2.0)), ("cauchy", dict()),
                     ("pareto", dict(b=3.0)), ("chi2", dict(df=3.0))]:
        qq = np.random.RandomState(3).random((3000, 1))[:, 0]
        assert_close(D(name, **kw).sample(3000, random_state=3), getattr(scipy.stats, name)(**kw).ppf(qq),
                     rtol=1e-10, atol=1e-13, what=f"Node.sample {name}")
    s = D("weibull_min", c=D("uniform", loc=1, scale=2)).sample(2000, random_state=4)
    qq = np.random.RandomState(4).random((2000, 2))
    # column order: ISNs take quantile columns in _id order, so the parameter
    # node uniform (created first) takes column 0 and weibull_min column 1
    ref = scipy.stats.weibull_min(c=scipy.stats.uniform(loc=1, scale=2).ppf(qq[:, 0])).ppf(qq[:, 1])
    assert_close(s, ref, rtol=1e-10, atol=1e-13, what="composite weibull_min column order")


def test_closed_form_correlated_iman_conover(gpu):
    """Closed-form distributions under ImanConover through Node.sample (modeling.py:571-583): the
    correlated samples equal the oracle's Iman-Conover (correlation.py:388-425 restated) applied to
    the same graph's uncorrelated samples (same random_state, same column assignment)."""
    from oracle.ic import iman_conover
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.modeling import NoOp

    C = np.array([[1.0, 0.5, -0.3], [0.5, 1.0, 0.2], [-0.3, 0.2, 1.0]])

    def graph():
        ds = [D("weibull_min", c=1.5), D("logistic", loc=2.0), D("gumbel_r", scale=0.5)]
        return ds, NoOp(*ds)

    n = 20_000
    ds, sink = graph()
    sink.sample(n, random_state=11)
    X = np.column_stack([d.samples_ for d in ds])
    ds, sink = graph()
    sink.correlate(*ds, corr_mat=C).sample(n, random_state=11)
    Y = np.column_stack([d.samples_ for d in ds])
    assert_close(Y, iman_conover(X, C)["Y"], rtol=1e-12, what="closed-form Iman-Conover")


# the fused native-LHS inverse CDF of the extended distributions (pbh_lhs_ppf -> k_ppf_ext with
# the generator inside the kernel): Node.sample(method="lhs") and row-offset windows against
# scipy's ppf on the same native-LHS quantiles (native.fill_lhs, the two-pass form)
_LHS_EXT = [("beta", dict(a=3.4, b=2.6, loc=0, scale=10)), ("beta", dict(a=0.5, b=0.5)),
            ("beta", dict(a=7.0, b=5.0, loc=-1.0, scale=3.0)), ("truncnorm", dict(a=-1.0, b=1.0, loc=2.0, scale=0.5)),
            ("truncnorm", dict(a=3.0, b=3.3)), ("binom", dict(n=20, p=0.3)), ("binom", dict(n=1000, p=0.7, loc=2)),
            ("bernoulli", dict(p=0.25))] + [c for c in _CLOSED[:30]] + [c for c in _CLOSED2[:48]]


@pytest.mark.parametrize("name,kw", _LHS_EXT)
def test_fused_lhs_ext_vs_scipy(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    n, s = 40_000, 21
    q = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = D(name, **kw).sample(n, method="lhs", random_state=s)
    if name in ("binom", "bernoulli"):
        np.testing.assert_array_equal(got, ref)
    else:
        assert_close(got, ref, rtol=1e-10, atol=1e-13, what=f"LHS {name} {kw}")
    # a window [row0, row0 + rows) of a 3-column design, column 2
    row0, rows = 12_345, 9_999
    q3 = native.fill_lhs(77, n, 3, row0=row0, nrows=rows)[:, 2]
    with np.errstate(all="ignore"):
        ref3 = getattr(scipy.stats, name)(**kw).ppf(q3)
    got3 = native.lhs_ppf(name, 77, n, 2, row0=row0, nrows=rows, **kw)
    if name in ("binom", "bernoulli"):
        np.testing.assert_array_equal(got3, ref3)
    else:
        assert_close(got3, ref3, rtol=1e-10, atol=1e-13, what=f"LHS window {name} {kw}")


def test_fused_lhs_pert_composite(gpu):
    """PERT (the reference's headline constructor, distributions.py:78-94 -> beta) with a
    composite mode under method="lhs": parameters per row, ISN columns in _id order."""
    import scipy.stats

    from probabilit_amd import distributions as dists
    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    n, s = 30_000, 5
    x = dists.PERT(0, 6, 10).sample(n, method="lhs", random_state=s)
    q = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    assert_close(x, scipy.stats.beta(a=3.4, b=2.6, loc=0, scale=10).ppf(q), what="PERT LHS")
    y = D("beta", a=D("uniform", loc=1, scale=3), b=2.0).sample(n, method="lhs", random_state=s)
    q2 = native.fill_lhs(seed_from(s), n, 2)
    a = scipy.stats.uniform(loc=1, scale=3).ppf(q2[:, 0])
    assert_close(y, scipy.stats.beta(a=a, b=2.0).ppf(q2[:, 1]), what="composite beta LHS")


def _ext_graph(kind):
    from probabilit_amd import distributions as dists
    from probabilit_amd.modeling import Distribution as D

    if kind == "pert":
        return [dists.PERT(0, 6, 10), dists.PERT(1, 2, 9, gamma=10), dists.PERT(-3, 0, 1), dists.PERT(5, 6, 7)]
    if kind == "discrete":
        return [D("binom", n=20, p=0.3), D("bernoulli", p=0.25), D("binom", n=1000, p=0.7, loc=2), D("norm")]
    return [D("truncnorm", a=-1.0, b=2.0, loc=1.0), D("weibull_min", c=1.7), D("logistic", loc=2.0),
            D("gumbel_r", scale=0.5), D("chi2", df=5.5), D("beta", 0.5, 0.5), D("lomax", c=1.88), D("gamma", a=2.0)]


@pytest.mark.parametrize("kind,n", [("pert", 50_000), ("discrete", 40_000), ("mixed", 30_001)])
def test_ext_generated_iman_conover(gpu, kind, n):
    """Extended distributions (PERT -> beta, truncnorm, binom, bernoulli, closed forms) correlated
    with method="lhs" go through the generated-column fast path (stratum-ordered generator + step-4
    regeneration, pbh_ppf_ext.hip): bit-identical to the general path fed the same native-LHS
    quantiles (sample_from_quantiles, X materialised and sorted), and that equals the oracle's
    Iman-Conover (correlation.py:388-425 restated) of the same uncorrelated samples."""
    from oracle.ic import iman_conover
    from probabilit_amd import native
    from probabilit_amd.modeling import NoOp
    from probabilit_amd.qmc import seed_from

    d = len(_ext_graph(kind))
    rng = np.random.default_rng(d)
    A = rng.normal(size=(d, d + 2))
    C = np.corrcoef(A)
    ds = _ext_graph(kind)
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    root.sample(n, random_state=9, method="lhs")
    fast = np.column_stack([x.samples_ for x in ds])
    q = native.fill_lhs(seed_from(9), n, d)
    root.sample_from_quantiles(q)
    general = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, general)
    ds = _ext_graph(kind)
    NoOp(*ds).sample_from_quantiles(q)
    X = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, iman_conover(X, C)["Y"])


# round 5: geom, randint, nbinom (exact) and invgamma, t (1e-10 relative):
# sampled, fused with the native LHS, and on the generated-column Iman-Conover path
_R5_DISCRETE = [("geom", dict(p=0.3)), ("geom", dict(p=0.02, loc=3)), ("geom", dict(p=1.0)),
                ("geom", dict(p=1e-6)), ("randint", dict(low=2, high=7)), ("randint", dict(low=-5, high=100, loc=1)),
                ("randint", dict(low=0, high=1)), ("randint", dict(low=2.5, high=7)),
                ("nbinom", dict(n=3.5, p=0.4)), ("nbinom", dict(n=20, p=0.9)),
                ("nbinom", dict(n=0.5, p=0.05, loc=2)), ("nbinom", dict(n=5, p=1.0)), ("nbinom", dict(n=100, p=0.3))]
_R5_CONT = [("invgamma", dict(a=2.5)), ("invgamma", dict(a=0.3, loc=1.0, scale=2.0)), ("invgamma", dict(a=60.0)),
            ("t", dict(df=1.0)), ("t", dict(df=2.5, loc=1.0, scale=3.0)), ("t", dict(df=0.4)), ("t", dict(df=30.0)),
            ("t", dict(df=1e4)), ("t", dict(df=3e7)), ("t", dict(df=np.inf)), ("t", dict(df=-1.0))]


@pytest.mark.parametrize("name,kw", _R5_DISCRETE + _R5_CONT)
def test_round5_distributions_ppf(gpu, name, kw):
    """The round-5 names against scipy's ppf on random and edge quantiles; discrete exactly
    (geom: numpy's log1p / expm1 ratio with scipy's one-step correction; randint: its closed
    form; nbinom: Boost's smallest k with I_p(n, k + 1) >= q), continuous to 1e-10 (t: scipy's
    stdtrit is cdflib's root search, itself within ~2.5e-11 of the quantile computed here)."""
    import scipy.stats

    from probabilit_amd import native

    q = np.concatenate([_q(20_000, 9), [-0.5, 1.5, np.nan]])
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = native.ppf(name, q, **kw)
    if name == "nbinom":
        # q = 1 - 2^-53: Boost's quantile (scipy) stops ~12 values past the answer in this far tail
        # (P(X > k) = 1.08e-16 at k = 670 for n = 0.5, p = 0.05, mpmath); the device returns the
        # definition there, the smallest k with P(X > k) <= 1 - q (scipy's own betainc decides)
        import scipy.special as sc

        edge = q == 1 - 2.0**-53
        k, n, p, loc = got[edge] - kw.get("loc", 0), kw["n"], kw["p"], kw.get("loc", 0)
        if p < 1.0:
            assert np.all(sc.betainc(k + 1, n, 1 - p) <= 2.0**-53) and np.all(sc.betainc(k, n, 1 - p) > 2.0**-53)
        got, ref = got[~edge], ref[~edge]
    if name in ("geom", "randint", "nbinom"):
        np.testing.assert_array_equal(got, ref)
    else:
        assert_close(got, ref, rtol=1e-10, atol=1e-13, what=f"{name} {kw}")


@pytest.mark.parametrize("name,kw", [c for c in _R5_DISCRETE + _R5_CONT if "2.5" not in str(c[1].get("low", ""))
                                     and c[1].get("df", 1.0) > 0])
def test_round5_fused_lhs(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    n, s = 30_000, 23
    q = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = D(name, **kw).sample(n, method="lhs", random_state=s)
    if name in ("geom", "randint", "nbinom"):
        np.testing.assert_array_equal(got, ref)
    else:
        assert_close(got, ref, rtol=1e-10, atol=1e-13, what=f"LHS {name} {kw}")


def test_round5_composite_parameters(gpu):
    """Per-row parameters (composite nodes, modeling.py:796-802) for every round-5 name."""
    import scipy.stats

    from probabilit_amd import native

    n = 8_000
    rng = np.random.default_rng(12)
    q = rng.random(n)
    p, a, df = 0.05 + 0.9 * rng.random(n), 0.5 + 5 * rng.random(n), 0.5 + 20 * rng.random(n)
    low = np.floor(rng.uniform(-10, 10, n))
    np.testing.assert_array_equal(native.ppf("geom", q, p=p), scipy.stats.geom(p).ppf(q))
    np.testing.assert_array_equal(native.ppf("randint", q, low=low, high=low + 7), scipy.stats.randint(low, low + 7).ppf(q))
    np.testing.assert_array_equal(native.ppf("nbinom", q, n=a, p=p), scipy.stats.nbinom(a, p).ppf(q))
    assert_close(native.ppf("invgamma", q, a=a), scipy.stats.invgamma(a).ppf(q), what="composite invgamma")
    assert_close(native.ppf("t", q, df=df), scipy.stats.t(df).ppf(q), what="composite t")


def test_round5_generated_iman_conover(gpu):
    """geom / randint / nbinom / invgamma / t correlated with method="lhs" take the generated-column
    path (discrete ones with their run heads): bit-identical to the general path on the same
    native quantiles, and equal to the oracle's Iman-Conover of the uncorrelated samples."""
    from oracle.ic import iman_conover
    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.modeling import NoOp
    from probabilit_amd.qmc import seed_from

    def graph():
        return [D("geom", p=0.3), D("randint", low=-3, high=40), D("nbinom", n=3.5, p=0.4), D("invgamma", a=2.5),
                D("t", df=4.0, loc=1.0), D("norm")]

    n, d = 40_000, 6
    C = np.corrcoef(np.random.default_rng(d).normal(size=(d, d + 2)))
    ds = graph()
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    root.sample(n, random_state=13, method="lhs")
    fast = np.column_stack([x.samples_ for x in ds])
    q = native.fill_lhs(seed_from(13), n, d)
    root.sample_from_quantiles(q)
    general = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, general)
    ds = graph()
    NoOp(*ds).sample_from_quantiles(q)
    X = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, iman_conover(X, C)["Y"])


def test_grouped_lhs_columns(gpu):
    """Uncorrelated native-LHS leaves outside the fused DAG kernel (an extended name in the
    graph) are drawn by one pbh_lhs_ppf_columns call, their table/guide setups spread over the
    step-4 lanes' streams: every column bit-identical to its own pbh_lhs_ppf (column index = the
    node's place in _id order, modeling.py:529-538), and a one-leaf graph is unchanged."""
    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.modeling import NoOp
    from probabilit_amd.qmc import seed_from

    spec = [("gamma", dict(a=2.5, scale=3.0)), ("poisson", dict(mu=30.0)), ("beta", dict(a=2.0, b=3.0)),
            ("binom", dict(n=20, p=0.3)), ("t", dict(df=4.0, loc=1.0)), ("norm", dict(loc=1.0, scale=2.0)),
            ("gamma", dict(a=0.7)), ("nbinom", dict(n=3.5, p=0.4)), ("lognorm", dict(s=0.5))]
    n, s = 50_001, 31
    ds = [D(name, **kw) for name, kw in spec]
    NoOp(*ds).sample(n, random_state=s, method="lhs")
    for col, ((name, kw), d) in enumerate(zip(spec, ds)):
        np.testing.assert_array_equal(d.samples_, native.lhs_ppf(name, seed_from(s), n, col, **kw), err_msg=name)
    one = D("beta", a=2.0, b=3.0)
    NoOp(one).sample(n, random_state=s, method="lhs")
    np.testing.assert_array_equal(one.samples_, native.lhs_ppf("beta", seed_from(s), n, 0, a=2.0, b=3.0))


def test_setup_table_cache(gpu):
    """Setup tables are kept per parameter set (pbh_table_cache.hip): a second sample with the
    same parameters is served from the cache and gives the same values; other parameters get
    tables of their own (no key collision)."""
    import ctypes

    from probabilit_amd import _lib, native

    def stats():
        e, b, h = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(_lib.load().pbh_table_cache_stats(ctypes.byref(e), ctypes.byref(b), ctypes.byref(h)))
        return e.value, b.value, h.value

    n = 20_000
    cases = [("gamma", dict(a=3.3)), ("poisson", dict(mu=17.5)), ("beta", dict(a=1.7, b=4.2)), ("binom", dict(n=33, p=0.2)),
             ("nbinom", dict(n=2.5, p=0.3)), ("chi", dict(df=4.5))]
    for name, kw in cases:
        first = native.lhs_ppf(name, 5, n, 1, **kw)
        e0, _, h0 = stats()
        again = native.lhs_ppf(name, 5, n, 1, **kw)
        e1, _, h1 = stats()
        np.testing.assert_array_equal(first, again, err_msg=name)
        assert e1 == e0 and h1 > h0, (name, e0, e1, h0, h1)
        bumped = dict(kw)
        key = next(iter(kw))
        bumped[key] = kw[key] * 1.25 if name not in ("binom",) else kw[key] + 1
        other = native.lhs_ppf(name, 5, n, 1, **bumped)
        assert stats()[0] == e1 + 1, name
        assert not np.array_equal(other, first), name


# round 6: more scipy.stats names, each against scipy's ppf (1e-10 relative,
# discrete exact), fused with the native LHS, per-row parameters and on the generated-column
# Iman-Conover path
_R6_CONT = [("trapz", dict(c=0.2, d=0.8)), ("johnsonsu", dict(a=2.55, b=2.25)),
            ("johnsonsu", dict(a=-1.0, b=0.5, loc=1.0, scale=2.0)), ("johnsonsb", dict(a=4.32, b=3.18)),
            ("johnsonsb", dict(a=-0.5, b=0.8)), ("powernorm", dict(c=4.45)), ("powernorm", dict(c=0.3)),
            ("laplace_asymmetric", dict(kappa=2.0)), ("laplace_asymmetric", dict(kappa=0.3, loc=1.0)),
            ("mielke", dict(k=10.4, s=4.6)), ("mielke", dict(k=0.7, s=2.0)), ("truncpareto", dict(b=2.0, c=5.0)),
            ("truncpareto", dict(b=0.5, c=1.5)), ("tukeylambda", dict(lam=3.13)), ("tukeylambda", dict(lam=0.0)),
            ("tukeylambda", dict(lam=-0.5)), ("gengamma", dict(a=4.42, c=-3.12)), ("gengamma", dict(a=1.5, c=2.0)),
            ("loggamma", dict(c=0.414)), ("loggamma", dict(c=5.0, scale=2.0)), ("dgamma", dict(a=1.1)),
            ("dgamma", dict(a=4.0, loc=-1.0)), ("f", dict(dfn=29, dfd=18)), ("f", dict(dfn=1.5, dfd=0.8)),
            ("f", dict(dfn=3.0, dfd=50.0, scale=0.5)), ("rdist", dict(c=1.6)), ("rdist", dict(c=8.0)),
            ("semicircular", dict()), ("betaprime", dict(a=5.0, b=6.0)), ("betaprime", dict(a=0.5, b=3.0)),
            ("johnsonsu", dict(a=1.0, b=-1.0)), ("truncpareto", dict(b=2.0, c=0.5)), ("gengamma", dict(a=1.0, c=0.0))]
# round 6, second set: pearson3, gennorm, halfgennorm, wrapcauchy, skewcauchy, moyal, kappa4, crystalball
_R6_CONT += [("pearson3", dict(skew=0.7)), ("pearson3", dict(skew=-1.3, loc=1.0)), ("pearson3", dict(skew=1e-6)),
             ("gennorm", dict(beta=1.3)), ("gennorm", dict(beta=0.5, scale=2.0)), ("halfgennorm", dict(beta=0.7)),
             ("halfgennorm", dict(beta=3.0)), ("wrapcauchy", dict(c=0.3)), ("wrapcauchy", dict(c=0.9)),
             ("skewcauchy", dict(a=0.4)), ("skewcauchy", dict(a=-0.7)), ("moyal", dict()),
             ("moyal", dict(loc=2.0, scale=0.5)), ("kappa4", dict(h=0.1, k=0.3)), ("kappa4", dict(h=-0.5, k=0.2)),
             ("kappa4", dict(h=0.0, k=-0.4)), ("kappa4", dict(h=0.3, k=0.0)), ("kappa4", dict(h=0.0, k=0.0)),
             ("crystalball", dict(beta=2.0, m=3.0)), ("crystalball", dict(beta=0.5, m=1.5))]
_R6_DISCRETE = [("dlaplace", dict(a=0.8)), ("dlaplace", dict(a=3.0, loc=2)), ("planck", dict(lambda_=0.51)),
                ("planck", dict(lambda_=3.0, loc=-1)), ("boltzmann", dict(lambda_=1.4, N=19)),
                ("boltzmann", dict(lambda_=0.1, N=200, loc=1))]


@pytest.mark.parametrize("name,kw", _R6_CONT + _R6_DISCRETE)
def test_round6_distributions_ppf(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native

    q = np.concatenate([_q(20_000, 31), np.linspace(0.01, 0.99, 2001), [-0.5, 1.5, np.nan]])
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = native.ppf(name, q, **kw)
    if name in ("dlaplace", "planck", "boltzmann"):
        np.testing.assert_array_equal(got, ref)
    else:
        if name == "mielke":
            # q = 1 - 2^-53: q^(s/k) is 1 - 4.9e-17, which rounds to 1.0 (glibc's pow and the device's
            # give 1.0, so qsk / (1 - qsk) = inf); numpy's SIMD power returns the double below 1, one
            # ulp off, and scipy's finite value follows from that ulp alone.  Either is accepted there.
            at = q == 1 - 2.0**-53
            assert np.all((got[at] == ref[at]) | np.isinf(got[at]))
            got, ref = got[~at], ref[~at]
        if name == "crystalball":
            # above pbeta x = ndtri(y), y = ndtr(-beta) + (q / N - C) / sqrt(2 pi) -> 1 as q -> 1: an ulp of
            # exp(-beta^2 / 2) (numpy's SIMD exp inside scipy, not libm's) moves y by ulps and x by
            # ulp(y) / pdf(x).  Where that exceeds the gate, allow 8 ulps of y, scaled by the conditioning.
            with np.errstate(all="ignore"):
                cond = 8 * np.spacing(1.0) / scipy.stats.norm.pdf(ref)
            ill = np.isfinite(ref) & (cond > 1e-10 * np.abs(ref)) & (q > 0.5)
            assert np.all(np.abs(got[ill] - ref[ill]) <= cond[ill]), (got[ill], ref[ill])
            got, ref = got[~ill], ref[~ill]
        assert_close(got, ref, rtol=1e-10, atol=1e-13, what=f"{name} {kw}")


@pytest.mark.parametrize("name,kw", _R6_CONT[:30] + _R6_CONT[33:] + _R6_DISCRETE)
def test_round6_fused_lhs_and_composite(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    n, s = 30_000, 29
    q = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = D(name, **kw).sample(n, method="lhs", random_state=s)
    exact = name in ("dlaplace", "planck", "boltzmann")
    if exact:
        np.testing.assert_array_equal(got, ref)
    else:
        assert_close(got, ref, rtol=1e-10, atol=1e-13, what=f"LHS {name} {kw}")
    # per-row (composite) loc: the same values shifted row by row
    loc = np.random.default_rng(3).integers(-3, 4, n).astype(float)
    kw2 = dict(kw, loc=loc + kw.get("loc", 0.0))
    with np.errstate(all="ignore"):
        ref2 = getattr(scipy.stats, name)(**kw2).ppf(q)
    got2 = native.ppf(name, q, **kw2)
    if exact:
        np.testing.assert_array_equal(got2, ref2)
    else:
        assert_close(got2, ref2, rtol=1e-10, atol=1e-12, what=f"composite {name} {kw}")


# round 6, third set: powerlognorm and jf_skew_t (closed forms on ndtri / the beta inverse), cosine,
# invgauss and wald (scipy: xsf's cosine_invcdf and Boost's quantile, solved here by Newton),
# foldcauchy (closed form) and foldnorm (Newton).  scipy's foldcauchy / foldnorm ppf is the generic
# brentq on _cdf (xtol 1e-14): where that cdf is flat to a few ulps (q within ~1e-12 of 0 or 1) its x
# is any of many; there the device x is accepted when scipy's own cdf maps it back onto q.
_R6_CONT3 = [("powerlognorm", dict(c=2.14, s=0.446)), ("powerlognorm", dict(c=0.5, s=1.5, loc=1.0)),
             ("jf_skew_t", dict(a=8.0, b=4.0)), ("jf_skew_t", dict(a=0.7, b=2.5, scale=2.0)),
             ("foldcauchy", dict(c=4.72)), ("foldcauchy", dict(c=0.0)), ("foldnorm", dict(c=1.95)),
             ("foldnorm", dict(c=0.0, scale=2.0)), ("cosine", dict()), ("cosine", dict(loc=1.0, scale=0.5)),
             ("invgauss", dict(mu=0.145)), ("invgauss", dict(mu=3.0)), ("invgauss", dict(mu=25.0)),
             ("wald", dict()), ("wald", dict(loc=-1.0, scale=2.0)), ("recipinvgauss", dict(mu=0.63)),
             ("recipinvgauss", dict(mu=4.0, loc=0.5)), ("exponnorm", dict(K=1.5)), ("exponnorm", dict(K=0.2, scale=3.0)),
             ("argus", dict(chi=1.0)), ("argus", dict(chi=4.0)), ("kstwobign", dict()), ("kstwobign", dict(loc=1.0)),
             ("rel_breitwigner", dict(rho=36.545)), ("rel_breitwigner", dict(rho=0.4, scale=2.0))]
_GENERIC_PPF = ("foldcauchy", "foldnorm", "recipinvgauss", "exponnorm", "argus", "rel_breitwigner")


def _check_third(name, kw, q, got, ref, what):
    import scipy.stats

    if name in _GENERIC_PPF:
        with np.errstate(all="ignore"):
            back = getattr(scipy.stats, name)(**kw).cdf(got)
        loose = (q < 1e-9) | (q > 1 - 1e-9)
        ok = loose & np.isfinite(got) & (np.abs(back - q) <= 4e-16 + 4 * np.spacing(q))
        got, ref = got[~ok], ref[~ok]
    assert_close(got, ref, rtol=1e-10, atol=1e-13, what=what)


@pytest.mark.parametrize("name,kw", _R6_CONT3)
def test_round6_third_set_ppf(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native

    m = 4_000 if name in _GENERIC_PPF else 20_000  # scipy's generic ppf runs brentq per quantile
    q = np.concatenate([_q(m, 37), np.linspace(0.01, 0.99, m // 10 + 1), [-0.5, 1.5, np.nan]])
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = native.ppf(name, q, **kw)
    _check_third(name, kw, q, got, ref, f"{name} {kw}")


@pytest.mark.parametrize("name,kw", _R6_CONT3)
def test_round6_third_set_fused_lhs_and_composite(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    n, s = (6_000 if name in _GENERIC_PPF else 30_000), 41
    q = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    with np.errstate(all="ignore"):
        ref = getattr(scipy.stats, name)(**kw).ppf(q)
    got = D(name, **kw).sample(n, method="lhs", random_state=s)
    _check_third(name, kw, q, got, ref, f"LHS {name} {kw}")
    loc = np.random.default_rng(5).integers(-3, 4, n).astype(float)
    kw2 = dict(kw, loc=loc + kw.get("loc", 0.0))
    with np.errstate(all="ignore"):
        ref2 = getattr(scipy.stats, name)(**kw2).ppf(q)
    got2 = native.ppf(name, q, **kw2)
    assert_close(got2, ref2, rtol=1e-10, atol=1e-12, what=f"composite {name} {kw}")


# round 6: betabinom and hypergeom, scipy's generic discrete ppf (the first k with cdf(k) >= q, cdf the
# sum of the pmf): exact, with scalar parameters (the CDF table) and per row (the per-draw sum)
_R6_DISCRETE3 = [("betabinom", dict(n=20, a=2.5, b=1.5)), ("betabinom", dict(n=200, a=0.6, b=3.0, loc=1)),
                 ("hypergeom", dict(M=50, n=12, N=20)), ("hypergeom", dict(M=500, n=300, N=150, loc=-2)),
                 ("nhypergeom", dict(M=40, n=12, r=8)), ("nhypergeom", dict(M=300, n=120, r=30, loc=1)),
                 ("yulesimon", dict(alpha=3.5)), ("yulesimon", dict(alpha=11.0, loc=-1))]


@pytest.mark.parametrize("name,kw", _R6_DISCRETE3)
def test_round6_summed_discrete_ppf(gpu, name, kw):
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    # (scipy's generic discrete ppf is a Python bisection per quantile: 6 000 of them per case)
    q = np.concatenate([_q(6_000, 43), np.linspace(0.01, 0.99, 601), [-0.5, 1.5, np.nan]])
    ref = getattr(scipy.stats, name)(**kw).ppf(q)
    np.testing.assert_array_equal(native.ppf(name, q, **kw), ref)
    # fused with the native LHS, and with a per-row loc (no table: the per-draw sum)
    n, s = 8_000, 47
    ql = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    np.testing.assert_array_equal(D(name, **kw).sample(n, method="lhs", random_state=s),
                                  getattr(scipy.stats, name)(**kw).ppf(ql))
    loc = np.random.default_rng(7).integers(-3, 4, n).astype(float)
    kw2 = dict(kw, loc=loc + kw.get("loc", 0.0))
    np.testing.assert_array_equal(native.ppf(name, ql, **kw2), getattr(scipy.stats, name)(**kw2).ppf(ql))


@pytest.mark.parametrize("kw", [dict(a=4.0), dict(a=-3.0, loc=1.0), dict(a=0.5, scale=2.0), dict(a=25.0),
                                dict(a=0.0)])
def test_skewnorm_ppf(gpu, kw):
    """skewnorm: scipy's ppf is Boost's quantile on its cdf Phi(x) - 2 T(x, a), whose left tail loses
    its relative precision for a > 0 (scipy's _cdf says so and patches it, its _ppf does not): compared
    at 1e-10 for q in [1e-6, 1 - 1e-6]; the edges as rv_continuous.ppf has them."""
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    q = np.concatenate([_q(20_000, 53), np.linspace(0.01, 0.99, 2001), [-0.5, 1.5, np.nan]])
    ref = scipy.stats.skewnorm(**kw).ppf(q)
    got = native.ppf("skewnorm", q, **kw)
    mid = (q >= 1e-6) & (q <= 1 - 1e-6)
    assert_close(got[mid], ref[mid], rtol=1e-10, atol=1e-13, what=f"skewnorm {kw}")
    edge = ~mid & ~((q > 0) & (q < 1))
    np.testing.assert_array_equal(got[edge], ref[edge])
    assert np.all(np.isfinite(got[~mid & (q > 0) & (q < 1)]))
    n, s = 30_000, 59
    ql = native.fill_lhs(seed_from(s), n, 1)[:, 0]
    lm = (ql >= 1e-6) & (ql <= 1 - 1e-6)
    got = D("skewnorm", **kw).sample(n, method="lhs", random_state=s)
    assert_close(got[lm], scipy.stats.skewnorm(**kw).ppf(ql[lm]), rtol=1e-10, atol=1e-13, what=f"LHS skewnorm {kw}")


@pytest.mark.parametrize("kw,m", [(dict(a=1.25, n=10), 3000), (dict(a=0.6, n=30, loc=2), 600), (dict(a=2.5, n=1000), 2000),
                                  (dict(a=0.0, n=7), 2000)])
def test_zipfian_ppf(gpu, kw, m):
    """zipfian: scipy's bisection on H(k, a) / H(n, a), exact (scipy's own ppf is a Python loop per q,
    so m quantiles per case)."""
    import scipy.stats

    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.qmc import seed_from

    q = np.concatenate([_q(m, 61), np.linspace(0.01, 0.99, 99), [-0.5, 1.5, np.nan]])
    np.testing.assert_array_equal(native.ppf("zipfian", q, **kw), scipy.stats.zipfian(**kw).ppf(q))
    ql = native.fill_lhs(seed_from(67), m, 1)[:, 0]
    np.testing.assert_array_equal(D("zipfian", **kw).sample(m, method="lhs", random_state=67),
                                  scipy.stats.zipfian(**kw).ppf(ql))


def test_round6_generated_iman_conover(gpu):
    """The round-6 names correlated with method="lhs" take the generated-column path (dlaplace /
    planck / boltzmann with their run heads): bit-identical to the general path on the same native
    quantiles, and equal to the oracle's Iman-Conover of the uncorrelated samples."""
    from oracle.ic import iman_conover
    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution as D
    from probabilit_amd.modeling import NoOp
    from probabilit_amd.qmc import seed_from

    def graph():
        return [D("johnsonsu", a=2.55, b=2.25), D("f", dfn=29, dfd=18), D("dgamma", a=1.1), D("dlaplace", a=0.8),
                D("planck", lambda_=0.51), D("boltzmann", lambda_=1.4, N=19), D("tukeylambda", lam=3.13),
                D("betaprime", a=5.0, b=6.0), D("semicircular"), D("trapz", c=0.2, d=0.8),
                D("pearson3", skew=0.7), D("gennorm", beta=1.3), D("halfgennorm", beta=0.7), D("wrapcauchy", c=0.3),
                D("skewcauchy", a=0.4), D("moyal"), D("kappa4", h=0.1, k=0.3), D("crystalball", beta=2.0, m=3.0),
                D("powerlognorm", c=2.14, s=0.446), D("jf_skew_t", a=8.0, b=4.0), D("foldcauchy", c=4.72),
                D("foldnorm", c=1.95), D("cosine"), D("invgauss", mu=0.145), D("wald"),
                D("betabinom", n=20, a=2.5, b=1.5), D("hypergeom", M=50, n=12, N=20), D("skewnorm", a=4.0),
                D("recipinvgauss", mu=0.63), D("exponnorm", K=1.5), D("argus", chi=1.0), D("kstwobign"),
                D("nhypergeom", M=40, n=12, r=8), D("yulesimon", alpha=3.5), D("zipfian", a=1.25, n=10),
                D("rel_breitwigner", rho=36.545)]

    n, d = 30_000, 36
    C = np.corrcoef(np.random.default_rng(d).normal(size=(d, d + 2)))
    ds = graph()
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    root.sample(n, random_state=17, method="lhs")
    fast = np.column_stack([x.samples_ for x in ds])
    q = native.fill_lhs(seed_from(17), n, d)
    root.sample_from_quantiles(q)
    general = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, general)
    ds = graph()
    NoOp(*ds).sample_from_quantiles(q)
    X = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, iman_conover(X, C)["Y"])
