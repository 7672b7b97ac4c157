"""Host half of the fused graph evaluation (probabilit_amd.dag.plan_graph): which graphs it
takes, the program it builds, its register allocation and the garbage collector's replay.
No device work: the plan is built from the graph alone (the kernel is tested in
tests/test_gpu_dag.py against the per-node path)."""

import networkx as nx
import numpy as np
import pytest

from probabilit_amd import _lib, dag
from probabilit_amd import modeling as m
from probabilit_amd.garbage_collector import GarbageCollector


class _Ev:
    def __init__(self, G, size=100):
        self.size = size
        self.slot = {nd: i for i, nd in enumerate(G.nodes)}


@pytest.fixture(autouse=True)
def _host_params(monkeypatch):
    # Distribution._params resolves Node parameters on the device; leaf scalars need no device
    monkeypatch.setattr(m.Distribution, "_params",
                        lambda self, n: [float(a) for a in m._parse_scipy_args(self.distr, self.args, self.kwargs)])


def _plan(sink, gc_strategy=None):
    G = sink.to_graph()
    order = list(nx.topological_sort(G))
    isns = sorted({n for n in sink.nodes() if n._is_initial_sampling_node()}, key=lambda n: n._id)
    gc = GarbageCollector(strategy=gc_strategy).set_sink(sink)
    return dag.plan_graph(order, isns, _Ev(G), gc), G


def _fund(years=20):
    r = 0
    for _ in range(years):
        r = r * m.Distribution("norm", loc=1.11, scale=0.15) + 1200
    return r


def _kinds(plan):
    return [o["kind"] for o in plan.ops]


def test_fund_program():
    plan, G = _plan(_fund())
    k = _kinds(plan)
    assert k.count(_lib.DAG_GEN) == 20 and k.count(_lib.DAG_BINARY) == 40 and len(k) == 60
    assert max(max(o["rd"], o["ra"], o["rb"]) for o in plan.ops) + 1 <= 2  # r and the year's draw
    # constants are immediates: every Add has b = ("imm", 1200.0)
    adds = [o for o in plan.ops if o["kind"] == _lib.DAG_BINARY and o["op"] == _lib.OPS["add"]]
    assert all(o["b"] == ("imm", 1200.0) and o["rb"] == -1 for o in adds)
    # gc_strategy=None keeps all 81 nodes, 60 of them vectors written by the kernel
    assert len(plan.kept) == 81 and len(plan.stored) == 60


def test_fund_gc_sink_only():
    sink = _fund()
    plan, _ = _plan(sink, gc_strategy=[])
    assert plan.kept == [sink] and plan.stored == [sink]
    assert sum(o["rd"] >= 0 for o in plan.ops if o["kind"] == _lib.DAG_BINARY) == 39  # the sink's add: store only


def test_flags_and_partials():
    a, b = m.Distribution("norm"), m.Distribution("uniform")
    s = m.Add(a, 1.0, b, 2.0)
    plan, G = _plan(s)
    ev_slot = _Ev(G).slot
    bins = [o for o in plan.ops if o["kind"] == _lib.DAG_BINARY]
    assert len(bins) == 3 and all(o["flag"] == ev_slot[s] for o in bins)  # every partial checked (:943-959)
    avg = m.Avg(a, b, 3.0)
    plan, G = _plan(avg)
    bins = [o for o in plan.ops if o["kind"] == _lib.DAG_BINARY]
    assert [o["flag"] is None for o in bins] == [True, True, False]  # k_average checks the mean only
    assert bins[-1]["op"] == _lib.OPS["truediv"] and bins[-1]["b"] == ("imm", 3.0)


def test_dead_draw_still_generated():
    a, dead = m.Distribution("norm"), m.Distribution("norm", scale=-1.0)
    plan, _ = _plan(m.NoOp(a + 1.0, dead), gc_strategy=[])
    assert sum(k == _lib.DAG_GEN for k in _kinds(plan)) == 2
    assert dead in plan.gen_nodes


@pytest.mark.parametrize("build", [
    lambda: m.Distribution("gamma", 2.0) + 1.0,  # no fused inverse CDF
    lambda: m.Distribution("norm") < 0.5,  # bool result
    lambda: m.Distribution("norm", loc=m.Distribution("uniform")) * 2.0,  # composite parameter
    lambda: m.Add(1.0, 2.0, m.Distribution("norm")),  # first partial is a numpy scalar
    lambda: m.Avg(1.0, 2.0, m.Distribution("norm")),  # Avg's first partial sum is a scalar too
    lambda: m.Abs(m.Constant(-1.0)) + m.Distribution("norm"),  # transform of a constant
    lambda: m.Add(*[d * 2.0 for d in [m.Distribution("norm", i) for i in range(20)]])
    + m.Multiply(*[m.Distribution("norm", i) for i in range(20)]),  # fits (each draw read once)
])
def test_declined_or_fused(build):
    plan, _ = _plan(build())
    fused = plan is not None
    sink = build()
    expect = isinstance(sink, m.Add) and len(sink.parents) == 2 and isinstance(sink.parents[1], m.Multiply)
    assert fused == expect


def test_too_many_live_values_declined():
    ds = [m.Distribution("norm", loc=float(i)) for i in range(20)]
    plan, _ = _plan(m.Add(*[d * 2.0 for d in ds]) + m.Multiply(*ds))
    assert plan is None  # all twenty draws live at once: more than 16 registers
    ds = [m.Distribution("norm", loc=float(i)) for i in range(12)]
    plan, _ = _plan(m.Add(*[d * 2.0 for d in ds]) + m.Multiply(*ds))
    assert plan is not None and max(o["rd"] for o in plan.ops) < _lib.DAG_MAX_REGS


def test_register_reuse_is_after_last_read():
    """A register freed by an op's last read may be that op's destination (the kernel reads
    its operands before writing), never an earlier live value's."""
    sink, _ = _mixed()
    plan, _ = _plan(sink)
    live = {}
    for i, o in enumerate(plan.ops):
        for r, name in ((o["ra"], "a"), (o["rb"], "b")):
            if r >= 0:
                assert live.get(r) == o[name][1], f"op {i} reads register {r} holding another value"
        if o["rd"] >= 0:
            live[o["rd"]] = o["dst"]


def _mixed():
    a = m.Distribution("norm", loc=1.0, scale=2.0)
    b = m.Distribution("uniform", loc=0.5, scale=3.0)
    c = m.Distribution("expon", scale=0.7)
    d = m.Distribution("lognorm", 0.4, scale=1.5)
    e = m.Distribution("triang", 0.3, loc=-1.0, scale=4.0)
    x = m.Add(a, b, 2.5, c)
    w = m.Max(m.Divide(m.Multiply(x, d) - e, m.Abs(c) + 1.0), a, 0.0) ** 0.5 + m.Mod(e, 1.25)
    v = m.Avg(m.Arctan2(w, b) + m.Exp(-m.Square(a) / 8), w, 1.5, a) + 2 ** m.Negate(c)
    return m.NoOp(v, m.Distribution("norm", 3.0)), np


def test_mixed_fits():
    plan, _ = _plan(_mixed()[0])
    assert plan is not None
    assert sum(k == _lib.DAG_GEN for k in _kinds(plan)) == 6


def test_loaded_vectors_alone_give_no_program(monkeypatch):
    """A NoOp over already sampled (correlated) vectors has nothing to compute: no kernel."""
    import torch

    ds = [m.Distribution("norm") for _ in range(3)]
    sink = m.NoOp(*ds)
    for d in ds:
        d.__dict__["_smp"] = torch.zeros(4, dtype=torch.float64)
    plan, _ = _plan(sink)
    assert plan is None
    s2 = m.NoOp(ds[0] * 2.0, ds[1])
    plan, _ = _plan(s2)
    assert [o["kind"] for o in plan.ops] == [_lib.DAG_LOAD, _lib.DAG_BINARY]
