"""Table-driven distribution nodes on the GPU (modeling.py:825-927) against the reference's
own numpy calls on the same quantiles (np.quantile / np.interp / searchsorted are the oracle:
the reference's _sample bodies), bit for bit, plus the reference's docstring pins."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _qs(n, seed):
    q = np.random.default_rng(seed).random(n)
    edge = np.array([0.0, 1e-300, 2.0 ** -53, 0.2, 0.5, 0.8, 1.0 - 2.0 ** -53, np.nextafter(1.0, 0)])
    return np.concatenate([q, edge])


@pytest.mark.parametrize("method", ["linear", "lower", "higher", "nearest", "midpoint"])
@pytest.mark.parametrize("data", [np.array([3.0]), np.array([5, 1, 4, 1, 5, 9, 2, 6]),
                                  np.random.default_rng(1).gamma(2.0, size=1001), np.arange(7) * 1.5])
def test_empirical_quantile(gpu, data, method):
    from probabilit_amd.modeling import EmpiricalDistribution

    q = _qs(5000, data.size)
    got = EmpiricalDistribution(data, method=method)._sample(q)
    ref = np.quantile(a=data, q=q, method=method)
    assert got.dtype == ref.dtype
    np.testing.assert_array_equal(got, ref)


@pytest.mark.parametrize("xp,fp", [([0, 0.2, 0.8, 1], [10, 15, 20, 25]), ([0.0, 1.0], [-3.0, 7.5]),
                                   (np.linspace(0, 1, 50), np.cumsum(np.random.default_rng(2).random(50)))])
def test_cumulative_interp(gpu, xp, fp):
    from probabilit_amd.modeling import CumulativeDistribution

    q = np.concatenate([_qs(5000, 3), np.asarray(xp, dtype=float)])
    np.testing.assert_array_equal(CumulativeDistribution(xp, fp)._sample(q), np.interp(x=q, xp=xp, fp=fp))


@pytest.mark.parametrize("values,p", [([10, 15, 20], [0.2, 0.3, 0.5]), ([1.5, -2.0], None),
                                      (list(range(37)), np.random.default_rng(5).dirichlet(np.ones(37)))])
def test_discrete_search(gpu, values, p):
    from probabilit_amd.modeling import DiscreteDistribution

    d = DiscreteDistribution(values, probabilities=p)
    q = _qs(5000, 4)
    q = q[q < np.cumsum(d.probabilities)[-1]]
    ref = d.values[np.searchsorted(np.cumsum(d.probabilities), v=q, side="right")]
    got = d._sample(q)
    assert got.dtype == ref.dtype
    np.testing.assert_array_equal(got, ref)


def test_discrete_out_of_range_raises_indexerror(gpu):
    from probabilit_amd.modeling import DiscreteDistribution

    d = DiscreteDistribution([1, 2], probabilities=[0.5, 0.5])
    with pytest.raises(IndexError):
        d._sample(np.array([0.3, 1.0]))


def test_docstring_pins_tables(gpu):
    """modeling.py:850-857 and 889-895."""
    from probabilit_amd.modeling import CumulativeDistribution, DiscreteDistribution

    distr = CumulativeDistribution([0, 0.2, 0.8, 1], [10, 15, 20, 25])
    np.testing.assert_allclose(distr._sample(np.linspace(0, 1, num=6)),
                               [10.0, 15.0, 16.66666667, 18.33333333, 20.0, 25.0], rtol=1e-9)
    np.testing.assert_allclose(distr.sample(9, random_state=42),
                               [16.45450099, 23.76785766, 19.43328285, 18.32215403, 13.90046601, 13.89986301,
                                11.4520903, 21.65440364, 18.3426251], rtol=1e-9)
    d = DiscreteDistribution([10, 15, 20], probabilities=[0.2, 0.3, 0.5])
    np.testing.assert_array_equal(d._sample(np.linspace(0, 1, num=5, endpoint=False)), [10, 15, 15, 20, 20])
    s = DiscreteDistribution(["A", "B", "C", "D", "E", "F"]).sample(9, random_state=42)
    np.testing.assert_array_equal(s, np.array(["C", "F", "E", "D", "A", "A", "A", "F", "D"]))


def test_tables_in_dag_with_lhs_and_correlation(gpu):
    """Table nodes inside a DAG: LHS columns are materialised for them, they take part in
    transforms and in Iman-Conover (step 4 reorders their sorted samples)."""
    from probabilit_amd.modeling import (CumulativeDistribution, DiscreteDistribution, Distribution,
                                         EmpiricalDistribution)

    e = EmpiricalDistribution(np.random.default_rng(0).normal(size=200))
    c = CumulativeDistribution([0, 0.5, 1], [0.0, 1.0, 4.0])
    k = DiscreteDistribution([1, 2, 3], [0.2, 0.3, 0.5])
    n = Distribution("norm")
    expr = e + c * k + n
    C = np.array([[1.0, 0.5, 0.2, 0.0], [0.5, 1.0, 0.1, 0.0], [0.2, 0.1, 1.0, 0.3], [0.0, 0.0, 0.3, 1.0]])
    expr.correlate(e, c, k, n, corr_mat=C)
    out = expr.sample(3000, random_state=1, method="lhs")
    np.testing.assert_allclose(out, e.samples_ + c.samples_ * k.samples_ + n.samples_, rtol=1e-12)
    # marginals preserved: sorted samples equal the uncorrelated sorted draws
    assert set(np.unique(k.samples_)) <= {1, 2, 3}
    Q = np.column_stack([np.sort(e.samples_), np.sort(c.samples_)])
    assert np.all(np.diff(Q, axis=0) >= 0)
