"""The DAG evaluator (Node.sample / sample_from_quantiles, modeling.py:431-614) on the GPU
against the reference's outputs on identical quantiles (tests/golden/dag.npz)."""

import numpy as np
import pytest

from conftest import assert_close, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dag():
    return golden("dag.npz")


def _fund():
    from probabilit_amd.modeling import Distribution

    nodes, r = [], 0
    for _ in range(20):
        i = Distribution("norm", loc=1.11, scale=0.15)
        nodes.append(i)
        r = r * i + 1200
    return r, nodes


def test_mutual_fund_sobol_quantiles(gpu, dag):
    r, nodes = _fund()
    sink = r.sample_from_quantiles(dag["fund_Q"])
    assert_close(np.column_stack([n.samples_ for n in nodes]), dag["fund_interest"], rtol=1e-10)
    assert_close(sink, dag["fund_sink"], rtol=1e-10)


def test_mutual_fund_sample_sobol_end_to_end(gpu, dag):
    """Node.sample(method='sobol') is bit-exact with scipy's engine, so the whole
    .sample() call reproduces the reference output for the same seed."""
    r, _ = _fund()
    sink = r.sample(4096, random_state=0, method="sobol")
    assert_close(sink, dag["fund_sink"], rtol=1e-10)


def test_readme_mutual_fund_pins(gpu, dag):
    """README.md:64-78 / tests/test_modeling.py:73-92 regression values."""
    r, _ = _fund()
    s = r.sample_from_quantiles(dag["fund999_Q"])
    np.testing.assert_allclose(s.mean(), 76583.58738496085, rtol=1e-12)
    np.testing.assert_allclose(s.std(), 33483.2245611436, rtol=1e-12)
    assert_close(s, dag["fund999_sink"], rtol=1e-10)


def test_readme_height(gpu, dag):
    from probabilit_amd.modeling import Distribution

    male = Distribution("norm", loc=176, scale=7.1)
    female = Distribution("norm", loc=162.5, scale=7.1)
    stat = male > female
    s = stat.sample_from_quantiles(dag["height_Q"])
    assert s.dtype == np.bool_
    np.testing.assert_array_equal(s, dag["height_sink"])
    assert s.mean() == 0.9039039039039038
    assert_close(male.samples_, dag["height_male"], rtol=1e-12)


def test_column_assignment(gpu, dag):
    from probabilit_amd.modeling import Distribution

    mu = Distribution("norm")
    a = Distribution("norm", loc=mu)
    b = Distribution("expon")
    e = a + b
    e.sample_from_quantiles(np.array([[0.1, 0.2, 0.3]]))
    got = np.array([mu.samples_[0], a.samples_[0], b.samples_[0], e.samples_[0]])
    assert_close(got, dag["colorder"], rtol=1e-12)


def test_expression_pow_mul_add(gpu, dag):
    from probabilit_amd.modeling import Distribution

    a = Distribution("norm", loc=5, scale=1)
    b = Distribution("expon", scale=1)
    expr = a ** b + a * b + 5 * b
    assert_close(expr.sample_from_quantiles(dag["expr_Q"]), dag["expr_sink"], rtol=1e-10)


def test_composite_parameters(gpu, dag):
    from probabilit_amd.modeling import Distribution

    g = Distribution("gamma", a=2.0, scale=3.0)
    p = Distribution("poisson", mu=g)
    m = Distribution("norm", loc=5.0, scale=1.0)
    s = Distribution("triang", c=0.4, loc=0.5, scale=1.0)
    n2 = Distribution("norm", loc=m, scale=s)
    root = p + n2 * 2 - 1
    out = root.sample_from_quantiles(dag["comp_Q"])
    got = np.column_stack([g.samples_, m.samples_, s.samples_, p.samples_, n2.samples_])
    assert_close(got, dag["comp_nodes"], rtol=1e-10)
    assert_close(out, dag["comp_sink"], rtol=1e-10)


@pytest.mark.parametrize("tag,d", [("corr8", 8), ("corr32", 32)])
def test_correlated_dag(gpu, dag, tag, d):
    """NoOp(*ds).correlate(*ds, C): ISN sampling + Iman-Conover.  The reorder is bit-exact
    (every column's ranks identical to the reference's); values inherit the ppf tolerance."""
    import scipy.stats

    from oracle.pipeline import cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    root = NoOp(*ds).correlate(*ds, corr_mat=dag[f"{tag}_C"])
    assert root.sample_from_quantiles(dag[f"{tag}_Q"]) is None
    Y = np.column_stack([x.samples_ for x in ds])
    ref = dag[f"{tag}_Y"]
    assert_close(Y, ref, rtol=1e-10)
    for k in range(d):
        np.testing.assert_array_equal(scipy.stats.rankdata(Y[:, k]), scipy.stats.rankdata(ref[:, k]))


def test_gc_strategy(gpu, dag):
    from probabilit_amd.modeling import Distribution, Exp

    a = Distribution("norm")
    inter = (a + a) ** 2 - a
    final = Exp(inter)
    out = final.sample_from_quantiles(np.array([[0.2], [0.5], [0.9]]), gc_strategy=[])
    assert_close(out, dag["gc_sink"], rtol=1e-12)
    assert [hasattr(a, "samples_"), hasattr(inter, "samples_")] == list(dag["gc_has"])
    final.sample_from_quantiles(np.array([[0.2], [0.5], [0.9]]), gc_strategy=[a])
    assert hasattr(a, "samples_") and not hasattr(inter, "samples_")


def test_constants_and_int_dtypes(gpu):
    from probabilit_amd.modeling import Add, Constant

    a = Constant(1)
    out = (a * 3 + 5).sample(5, random_state=0)
    assert out.dtype == np.int64 and list(out) == [8] * 5
    assert list(Add(10, 5, 5).sample(5, random_state=0)) == [20] * 5


def test_dice_equal_lhs(gpu):
    from probabilit_amd.modeling import Distribution, Equal

    d1 = Distribution("uniform", loc=1, scale=6) // 1
    d2 = Distribution("uniform", loc=1, scale=6) // 1
    s = Equal(d1, d2).sample(60_000, random_state=42, method="lhs")
    assert s.dtype == np.bool_
    assert abs(s.mean() - 1 / 6) < 0.01


def test_native_lhs_sample_reproducible(gpu):
    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(8)]
    root = NoOp(*ds).correlate(*ds, corr_mat=cfg3_corr(8))
    root.sample(50_000, random_state=3, method="lhs")
    first = np.column_stack([x.samples_ for x in ds])
    root.sample(50_000, random_state=3, method="lhs")
    np.testing.assert_array_equal(np.column_stack([x.samples_ for x in ds]), first)


@pytest.mark.parametrize("d,n", [(8, 300_001), (32, 65_536), (3, 10)])
def test_lhs_generated_fast_path_matches_materialized(gpu, d, n):
    """sample(method='lhs') hands correlated ISNs to Iman-Conover as generators (stratum-
    ordered generation, ranks from the permutation, no X sort).  It must equal the general
    path fed the same native-LHS quantile matrix bit for bit."""
    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd import native
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    root = NoOp(*ds).correlate(*ds, corr_mat=cfg3_corr(d))
    root.sample(n, random_state=77, method="lhs")
    fast = np.column_stack([x.samples_ for x in ds])
    root.sample_from_quantiles(native.fill_lhs(77, n, d))
    general = np.column_stack([x.samples_ for x in ds])
    np.testing.assert_array_equal(fast, general)


def test_non_finite_raises(gpu):
    from probabilit_amd.modeling import Distribution, Log

    with pytest.raises(ValueError, match="non-finite"):
        Log(Distribution("norm")).sample(100, random_state=0)


def test_unsupported_distribution_fails_loudly(gpu):
    from probabilit_amd.modeling import Distribution

    # a scipy name with no device kernel: the message names the supported set
    with pytest.raises(NotImplementedError, match=r"no native inverse-CDF kernel.*'weibull_min'"):
        Distribution("vonmises", kappa=2.0).sample(10, random_state=0)
    with pytest.raises(AttributeError):
        Distribution("no_such_distribution").sample(10, random_state=0)


def test_int_negative_power(gpu):
    from probabilit_amd.modeling import Constant, Distribution

    x = (Distribution("poisson", mu=3) + 1) ** Constant(-1)
    assert x.sample(10, random_state=0).dtype == np.float64  # float ** int is fine
    with pytest.raises(ValueError, match="negative integer powers"):
        (Constant(2) ** Constant(-1)).sample(3, random_state=0)
    with pytest.raises(ValueError, match="non-finite"):
        (Distribution("poisson", mu=3) ** Constant(-1)).sample(1000, random_state=0)  # 0 ** -1 = inf


def test_graph_plan_reused_and_invalidated(gpu):
    """Node._plan keeps an evaluation's graph analysis between calls; a correlation added with
    correlate(), a copy() and a new node on top each get an analysis of their own graph, so every
    result equals a fresh graph's."""
    from probabilit_amd.modeling import Distribution, NoOp

    def fresh(corr):
        a, b = Distribution("norm", loc=1, scale=2), Distribution("gamma", a=2.0)
        root = NoOp(a, b)
        if corr:
            root.correlate(a, b, corr_mat=np.array([[1.0, 0.6], [0.6, 1.0]]))
        root.sample(5000, random_state=3, method="lhs")
        return a.samples_.copy(), b.samples_.copy()

    a, b = Distribution("norm", loc=1, scale=2), Distribution("gamma", a=2.0)
    root = NoOp(a, b)
    root.sample(5000, random_state=3, method="lhs")
    plan = root.__dict__["_plan_cache"][1]
    root.sample(5000, random_state=3, method="lhs")
    assert root.__dict__["_plan_cache"][1] is plan  # reused
    ref = fresh(False)
    np.testing.assert_array_equal(a.samples_, ref[0])
    root.correlate(a, b, corr_mat=np.array([[1.0, 0.6], [0.6, 1.0]]))
    root.sample(5000, random_state=3, method="lhs")
    assert root.__dict__["_plan_cache"][1] is not plan
    ref = fresh(True)
    np.testing.assert_array_equal(a.samples_, ref[0])
    np.testing.assert_array_equal(b.samples_, ref[1])
    dup = root.copy()  # (a copied correlated graph keeps deep copies of its correlation's nodes, as the
    assert "_plan_cache" not in dup.__dict__  # reference's copy() does: sampling one is not defined)
    plain_root = NoOp(a2 := Distribution("norm", loc=1, scale=2), Distribution("gamma", a=2.0))
    plain_root.sample(5000, random_state=3, method="lhs")
    dup2 = plain_root.copy()
    dup2.sample(5000, random_state=3, method="lhs")
    np.testing.assert_array_equal(list(dup2.get_parents())[0].samples_, a2.samples_)
    top = a * 2.0 + b  # a new graph over the same leaves, without root's correlation
    out = top.sample(5000, random_state=3, method="lhs")
    plain = fresh(False)
    np.testing.assert_array_equal(a.samples_, plain[0])
    np.testing.assert_array_equal(out, plain[0] * 2.0 + plain[1])
