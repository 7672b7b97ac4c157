"""Fused evaluation of elementwise graphs: the per-node loop of Node.sample
(modeling.py:586-612) compiled into one straight-line program and run by one kernel
(pbh_dag_eval, csrc/pbh_dag.hip).

A graph qualifies when every node is
  * a leaf Distribution with scalar parameters whose inverse CDF has a fused form (norm,
    uniform, expon, lognorm, triang) and that is not yet sampled -- a GEN op on its quantile
    column (native LHS, Sobol' or any quantile vector), or
  * a node already sampled into a float64 device vector (the correlated variables, after the
    correlator ran) -- a LOAD op, or
  * a Constant (an immediate operand), or
  * an Add / Multiply / Max / Min / Avg / NoOp, a float64 BinaryTransform (Subtract, Divide,
    FloorDivide, Mod, Power, Arctan2) or any UnaryTransform,
and no Transform has only Constant operands (those stay numpy scalars).  Other graphs take the
per-node path unchanged.  Within a fused graph every value is computed by the same inline
functions as the per-node kernels, so samples are bit-identical; the garbage collector's
decisions are replayed on the host (GarbageCollector.freed_by) and only the nodes it keeps are
written to HBM, so with gc_strategy=[] the intermediate nodes never leave the chip.  Each
node's non-finite flag word is set exactly as by its own kernel (a Variadic node's partial
results included, :943-959), so the error raised afterwards is the same.
"""

import ctypes
import os

from . import _lib, device

GEN_DISTS = {"norm", "uniform", "expon", "lognorm", "triang"}
_BINARY = {"add", "sub", "mul", "truediv", "floordiv", "mod", "pow", "max", "min", "arctan2"}


def enabled():
    """PBH_DAG=0 selects the per-node path (A/B measurements and the fused-vs-unfused tests)."""
    return os.environ.get("PBH_DAG", "1") != "0"


counts = {"fused": 0, "declined": 0}  # evaluations that took / did not take the fused kernel


class _Unfusable(Exception):
    pass


class _Plan:
    """Abstract program over node keys, then registers."""

    def __init__(self, n, ev):
        self.n = n
        self.ev = ev
        self.ops = []  # dicts: kind, op, dst, a, b, flag, store, value, params, node
        self.val = {}  # node -> ("imm", float) | ("key", key)
        self.emitted = set()
        self.gens = []  # GEN nodes in emission order
        self.loads = []  # (node, tensor) LOAD inputs
        self.need = {}  # node -> Sethi-Ullman register need

    def add(self, kind, dst=None, a=None, b=None, op=0, flag=None, value=0.0, params=(0.0, 0.0, 0.0), node=None):
        self.ops.append(dict(kind=kind, op=op, dst=dst, a=a, b=b, flag=flag, store=None, value=value,
                             params=tuple(params), node=node))
        return len(self.ops) - 1


def _scalar(value, n):
    from .modeling import _Broadcast

    bc = value if isinstance(value, _Broadcast) else _Broadcast(value, n)
    return float(bc.value)


def _classify(plan, node, isns):
    """Record node's value: an immediate, a lazily emitted leaf, or its transform ops."""
    import numpy as np

    from .modeling import (Avg, BinaryTransform, Constant, Distribution, NoOp, UnaryTransform, VariadicTransform,
                           _Broadcast, _dtype_of)

    n = plan.n
    dev = node.__dict__.get("_smp", None) if "_smp" in node.__dict__ else None
    if "_smp" in node.__dict__:  # sampled before (correlated variables, ISN ancestors)
        if dev is None:
            plan.val[node] = ("none",)
        elif isinstance(dev, _Broadcast):
            if dev.dtype not in (np.float64, np.int64, np.bool_):
                raise _Unfusable
            plan.val[node] = ("imm", _scalar(dev, n))
        else:
            if _dtype_of(dev) != np.float64:
                raise _Unfusable
            plan.val[node] = ("leaf", "load", dev)
            plan.need[node] = 1
        return
    if isinstance(node, Constant):
        try:
            plan.val[node] = ("imm", _scalar(node.value, n))
        except (TypeError, ValueError):
            raise _Unfusable
        return
    if type(node) is Distribution:
        if node not in isns or node.distr not in GEN_DISTS or not node.is_leaf:
            raise _Unfusable
        params = node._params(n)
        if not all(isinstance(p, float) for p in params):
            raise _Unfusable
        plan.val[node] = ("leaf", "gen", params)
        plan.need[node] = 1
        return
    if isinstance(node, NoOp):
        plan.val[node] = ("none",)
        return
    if isinstance(node, (Avg, VariadicTransform, BinaryTransform, UnaryTransform)):
        if isinstance(node, VariadicTransform) and not isinstance(node, Avg):
            if node.op_name not in ("add", "mul", "max", "min") or len(node.parents) < 2:
                raise _Unfusable  # (reduce of one parent: that parent's own samples)
        if isinstance(node, BinaryTransform) and node.op_name not in _BINARY:
            raise _Unfusable
        vals = [plan.val[p][0] for p in node.get_parents()]
        if "none" in vals:
            raise _Unfusable  # NoOp's samples are None: arithmetic on it raises in the reference
        if all(v == "imm" for v in vals):
            raise _Unfusable  # a numpy scalar result: the per-node path keeps it on the host
        ops = list(node.get_parents())
        if len(ops) >= 2 and all(plan.val[p][0] == "imm" for p in ops[:2]):
            # the first partial of the reduce (Avg's running sum too) is a scalar: the op has one
            # immediate slot, so this shape stays on the per-node path
            raise _Unfusable
        plan.val[node] = ("xform",)
        plan.need[node] = _need(plan, node)
        return
    raise _Unfusable


def _need(plan, node):
    """Registers to evaluate node's expression tree (Sethi-Ullman, sharing ignored)."""
    needs = [plan.need.get(p, 0) for p in node.get_parents()]
    if len(needs) == 1:
        return max(needs[0], 1)
    from .modeling import VariadicTransform

    if isinstance(node, VariadicTransform):  # reduced in order: the accumulator plus the next parent
        return max([needs[0]] + [1 + x for x in needs[1:]] + [1])
    hi, lo = max(needs), min(needs)
    return max(hi, lo + 1, 1)


def _emit(plan, node):
    """Emit node's ops after its operands' (depth first, the costlier operand of a binary op
    first), so that few values are live at once."""
    from .modeling import Avg, BinaryTransform, NoOp, UnaryTransform, VariadicTransform

    if node in plan.emitted:
        return
    v = plan.val[node]
    if v[0] == "leaf":
        _emit_leaf(plan, node)
        return
    if v[0] != "xform":
        if isinstance(node, NoOp):  # no value: its parents are evaluated, loaded vectors left alone
            plan.emitted.add(node)
            for p in node.parents:
                if plan.val[p][:2] != ("leaf", "load"):
                    _emit(plan, p)
        return
    plan.emitted.add(node)
    flag = plan.ev.slot[node]
    if isinstance(node, Avg):  # k_average: s = p0 + p1 + ..., x = s / m, only x checked
        parts = list(node.parents)
        acc = _operand(plan, parts[0])
        for j, p in enumerate(parts[1:]):
            b = _operand(plan, p)
            key = ("tmp", node, j)
            plan.add(_lib.DAG_BINARY, dst=key, a=acc, b=b, op=_lib.OPS["add"], node=node)
            acc = ("key", key)
        plan.add(_lib.DAG_BINARY, dst=node, a=acc, b=("imm", float(len(parts))), op=_lib.OPS["truediv"], flag=flag,
                 node=node)
    elif isinstance(node, VariadicTransform):  # functools.reduce, each partial flagged (:943-959)
        parts = list(node.parents)
        acc = _operand(plan, parts[0])
        for j, p in enumerate(parts[1:]):
            b = _operand(plan, p)
            key = node if j == len(parts) - 2 else ("tmp", node, j)
            plan.add(_lib.DAG_BINARY, dst=key, a=acc, b=b, op=_lib.OPS[node.op_name], flag=flag, node=node)
            acc = ("key", key)
    elif isinstance(node, BinaryTransform):
        pa, pb = node.parents
        for p in sorted((pa, pb), key=lambda q: -plan.need.get(q, 0)):
            _operand(plan, p)
        plan.add(_lib.DAG_BINARY, dst=node, a=_operand(plan, pa), b=_operand(plan, pb), op=_lib.OPS[node.op_name],
                 flag=flag, node=node)
    else:
        assert isinstance(node, UnaryTransform)
        plan.add(_lib.DAG_UNARY, dst=node, a=_operand(plan, node.parent), op=_lib.OPS[node.op_name], flag=flag,
                 node=node)


def _emit_leaf(plan, node):
    if node in plan.emitted:
        return
    plan.emitted.add(node)
    v = plan.val[node]
    if v[1] == "gen":
        p = list(v[2]) + [0.0] * (3 - len(v[2]))
        plan.add(_lib.DAG_GEN, dst=node, op=_lib.DIST_IDS[node.distr], flag=plan.ev.slot[node], params=p, node=node)
        plan.gens.append(node)
    else:
        plan.add(_lib.DAG_LOAD, dst=node, node=node)
        plan.loads.append((node, v[2]))


def _operand(plan, node):
    v = plan.val[node]
    if v[0] == "imm":
        return v
    if v[0] == "none":
        raise _Unfusable  # NoOp's samples are None: arithmetic on it raises in the reference
    _emit(plan, node)
    return ("key", node)


def _allocate(plan):
    """Registers for the keys, freed after their last use; None if more than DAG_MAX_REGS."""
    last = {}
    for i, o in enumerate(plan.ops):
        for opnd in (o["a"], o["b"]):
            if opnd is not None and opnd[0] == "key":
                last[opnd[1]] = i
    free = list(range(_lib.DAG_MAX_REGS))[::-1]
    reg = {}
    used = 0
    for i, o in enumerate(plan.ops):
        ra = rb = -1
        for name in ("a", "b"):
            opnd = o[name]
            if opnd is not None and opnd[0] == "key":
                r = reg[opnd[1]]
                if name == "a":
                    ra = r
                else:
                    rb = r
        o["ra"], o["rb"] = ra, rb
        for opnd in (o["a"], o["b"]):
            if opnd is not None and opnd[0] == "key" and last[opnd[1]] == i and opnd[1] in reg:
                free.append(reg.pop(opnd[1]))
        key = o["dst"]
        needs = key is not None and (last.get(key, -1) > i or o["kind"] == _lib.DAG_GEN)
        if needs:
            if not free:
                return None
            r = free.pop()
            used = max(used, r + 1)
            o["rd"] = r
            if last.get(key, -1) > i:
                reg[key] = r
            else:
                free.append(r)
        else:
            o["rd"] = -1
    return used


def plan_graph(order, isns, ev, gc):
    """The fused program for the graph whose nodes are `order` (topological), or None when
    the graph is outside the fused subset.  Host-only (no device work): the plan's ops carry
    registers (rd / ra / rb), and plan.kept / plan.freed / plan.stored / plan.gen_nodes say
    which nodes keep samples, which the collector frees, which the kernel writes, and which
    draws it makes (one quantile column each, in ISN order)."""
    plan = _Plan(ev.size, ev)
    try:
        for node in order:
            _classify(plan, node, isns)
        _emit(plan, order[-1])  # the sink: the only node without children
        for nd in isns:  # every draw is made (and flagged) even when nothing reads or keeps it
            if plan.val[nd][:2] == ("leaf", "gen"):
                _emit_leaf(plan, nd)
        if not plan.ops or _allocate(plan) is None:
            return None
    except (_Unfusable, RecursionError):
        return None
    plan.gen_nodes = [nd for nd in isns if plan.val[nd][:2] == ("leaf", "gen")]
    if len(plan.gen_nodes) != sum(1 for nd in isns if "_smp" not in nd.__dict__):
        return None
    plan.freed = gc.freed_by(order)
    plan.kept = [nd for nd in order if nd not in plan.freed]
    plan.stored = [nd for nd in plan.kept if plan.val[nd][0] == "xform" or plan.val[nd][:2] == ("leaf", "gen")]
    return plan


def try_evaluate(order, isns, source, ev, gc):
    """Evaluate the graph whose nodes are `order` (topological) with one fused kernel.

    Returns False (nothing consumed from `source`, no node touched) when the graph is outside
    the fused subset; otherwise assigns samples the way the per-node loop plus the garbage
    collector would leave them and returns True."""
    if not enabled():
        return False
    from .modeling import Constant, NoOp, _Broadcast

    n = ev.size
    plan = plan_graph(order, isns, ev, gc)
    if plan is None:
        counts["declined"] += 1
        return False
    gen_nodes, freed = plan.gen_nodes, plan.freed

    # ---- commit: quantile columns in ISN order (modeling.py:529-538), outputs, launch
    cols = {nd: source.next_column() for nd in gen_nodes}
    srcs, keep_alive, row0 = [], [], None
    src_index = {}
    for nd in plan.gens:
        c = cols[nd]
        s = _lib.DagSource()
        if c[0] == "lhs":
            _, seed, n_total, col, r0 = c
            s.kind, s.seed, s.n_total, s.col = _lib.QSRC_LHS, seed, n_total, col
            row0 = r0
        elif c[0] == "sobol":
            _, src, col = c
            sv = [int(x) for x in src.sv[col]]
            s.kind, s.bits, s.shift = _lib.QSRC_SOBOL, int(src.bits), int(src.shift[col])
            for b, x in enumerate(sv):
                s.sv[b] = x
            row0 = src.row0
        else:
            _, q, stride = c
            s.kind, s.q, s.stride = _lib.QSRC_VECTOR, q.data_ptr(), int(stride)
            keep_alive.append(q)
        src_index[nd] = len(srcs)
        srcs.append(s)
    vectors, vindex = [], {}
    for nd, t in plan.loads:
        vindex[("in", nd)] = len(vectors)
        vectors.append(t)
    outputs = {}
    for nd in plan.stored:
        outputs[nd] = device.empty(n)
        vindex[("out", nd)] = len(vectors)
        vectors.append(outputs[nd])
    ops = (_lib.DagOp * len(plan.ops))()
    for i, o in enumerate(plan.ops):
        d = ops[i]
        d.kind, d.op, d.dst, d.a, d.b = o["kind"], o["op"], o["rd"], o["ra"], o["rb"]
        d.flag = o["flag"] if o["flag"] is not None else -1
        imm = [x[1] for x in (o["a"], o["b"]) if x is not None and x[0] == "imm"]
        d.value = imm[0] if imm else 0.0
        for j in range(3):
            d.params[j] = o["params"][j]
        d.src = -1
        if o["kind"] == _lib.DAG_GEN:
            d.src = src_index[o["node"]]
        elif o["kind"] == _lib.DAG_LOAD:
            d.src = vindex[("in", o["node"])]
        d.store = -1
        if o["dst"] is o["node"] and ("out", o["node"]) in vindex:
            d.store = vindex[("out", o["node"])]
    vec_arr = (ctypes.c_void_p * max(len(vectors), 1))(*[t.data_ptr() for t in vectors])
    src_arr = (_lib.DagSource * max(len(srcs), 1))(*srcs)
    _lib.check(_lib.load().pbh_dag_eval(ops, len(plan.ops), src_arr, len(srcs), vec_arr, len(vectors),
                                        0 if row0 is None else int(row0), n, ev.flags.data_ptr(), device.stream()),
               "fused graph")
    del keep_alive

    # ---- the state the per-node loop and the garbage collector would leave
    for nd in order:
        if nd in freed:
            if "_smp" in nd.__dict__:
                del nd.samples_
            continue
        if nd in outputs:
            nd._set_device(outputs[nd])
        elif "_smp" in nd.__dict__:
            continue
        elif isinstance(nd, Constant):
            nd._set_device(_Broadcast(nd.value, n))
        elif isinstance(nd, NoOp):
            nd._set_device(None)
    counts["fused"] += 1
    return True
