"""Drop-in for probabilit.modeling (tommyod/probabilit @ 2025-09-19, src/probabilit/modeling.py).

The modeling language is unchanged: Node / Constant / Distribution / Transform classes with
overloaded operators build a lazy DAG, `Node.sample(size, random_state, method, correlator,
gc_strategy)` draws quantiles and `Node.sample_from_quantiles(quantiles, ...)` evaluates the
graph.  What changes is where the numbers live and who computes them:

* every node's samples are a device vector in HBM (torch-allocated, `cuda:<LOCAL_RANK>`);
  `node.samples_` is a numpy view materialised lazily on first access (one D2H copy);
* quantile columns come from GPU generators (probabilit_amd.qmc), the inverse CDFs from
  HIP kernels (pbh_ppf / fused pbh_lhs_ppf), transforms from pbh_elementwise, and the
  Iman-Conover reorder from pbh_iman_conover;
* Constants stay scalars until someone reads `.samples_` (Constant._sample of :760-763 is
  an `np.ones(size) * value` broadcast; no kernel needs it materialised);
* the non-finite check of :600-606 is fused into the producing kernels (one device flag
  per node, read once at the end; the first offending node in topological order raises).

Node-visiting order, quantile-column assignment (initial sampling nodes by creation id,
then the rest in networkx topological order), correlation validation, garbage collection
and the errors raised follow the reference line by line (citations below).
"""

import abc
import copy
import ctypes
import functools
import itertools
import numbers
import warnings

import networkx as nx
import numpy as np
import scipy.stats

from . import _lib, dag, device, qmc
from .correlation import Cholesky, ImanConover, PermutationCorrelator, nearest_correlation_matrix
from .garbage_collector import GarbageCollector
from .utils import build_corrmat

__all__ = ["Node", "Constant", "Distribution", "EmpiricalDistribution", "CumulativeDistribution",
           "DiscreteDistribution", "Transform", "VariadicTransform", "BinaryTransform", "UnaryTransform",
           "NoOp", "Avg", "scalar_transform", "MultivariateDistribution", "MarginalDistribution"]


def python_to_prob(argument):
    """Numbers become Constants, Nodes pass through (modeling.py:272-279)."""
    if isinstance(argument, numbers.Number):
        return Constant(argument)
    if isinstance(argument, Node):
        return argument
    raise ValueError(f"Type not compatible with probabilit: {argument}")


# =============================================================================
# device sample containers
# =============================================================================
_PBH_DTYPE = {np.dtype(bool): _lib.BOOL, np.dtype(np.int64): _lib.INT64, np.dtype(np.float64): _lib.FLOAT64}


def _canonical(dt):
    """The device dtype used for numpy dtype `dt` (bool / int64 / float64)."""
    dt = np.dtype(dt)
    if dt == np.bool_:
        return np.dtype(bool)
    if np.issubdtype(dt, np.integer):
        return np.dtype(np.int64)
    if np.issubdtype(dt, np.floating):
        return np.dtype(np.float64)
    raise TypeError(f"probabilit_amd: samples of dtype {dt} are not supported on the device")


class _Broadcast:
    """A Constant's `np.ones(size, dtype=type(value)) * value` kept as a scalar."""

    __slots__ = ("value", "n", "dtype")

    def __init__(self, value, n, dtype=None):
        self.dtype = _canonical(np.dtype(type(value)) if dtype is None else dtype)
        self.value = self.dtype.type(value)
        self.n = int(n)

    def host(self):
        return np.full(self.n, self.value, dtype=self.dtype)

    def operand(self):
        v = self.value
        if self.dtype == np.float64:
            return _lib.Operand(None, _lib.FLOAT64, float(v), 0)
        return _lib.Operand(None, _PBH_DTYPE[self.dtype], float(v), int(v))


def _dtype_of(x):
    if isinstance(x, _Broadcast):
        return x.dtype
    import torch

    return {torch.float64: np.dtype(np.float64), torch.int64: np.dtype(np.int64),
            torch.bool: np.dtype(bool)}[x.dtype]


def _operand(x):
    if isinstance(x, _Broadcast):
        return x.operand()
    return _lib.Operand(x.data_ptr(), _PBH_DTYPE[_dtype_of(x)], 0.0, 0)


def _to_device_samples(value):
    import torch

    if value is None or isinstance(value, _Broadcast):
        return value
    if isinstance(value, torch.Tensor):
        return value
    a = np.asarray(value)
    return device.to_device(a.astype(_canonical(a.dtype), copy=False))


def _alloc(n, dt):
    return device.empty(n, _canonical(dt).name)


def _as_float_vector(x, n):
    """float64 device vector or python float for a distribution parameter."""
    if isinstance(x, _Broadcast):
        return float(x.value)
    if _dtype_of(x) == np.float64:
        return x
    return _elementwise("cast", x, None, n, np.dtype(np.float64), np.dtype(np.float64), flag=None)


class _Evaluation:
    """Per-sample() state: one non-finite flag per node, the current size."""

    def __init__(self, size, nodes):
        self.size = size
        self.slot = {node: i for i, node in enumerate(nodes)}
        self.flags = device.zeros(max(len(nodes), 1), "int32")

    def flag_ptr(self, node):
        return self.flags.data_ptr() + 4 * self.slot[node]


# =============================================================================
# device kernels behind the Transform nodes
# =============================================================================
_NP_BINARY = {"add": np.add, "sub": np.subtract, "mul": np.multiply, "truediv": np.true_divide,
              "floordiv": np.floor_divide, "mod": np.mod, "pow": np.power, "max": np.maximum,
              "min": np.minimum, "and": np.logical_and, "or": np.logical_or, "eq": np.equal,
              "ne": np.not_equal, "lt": np.less, "le": np.less_equal, "gt": np.greater,
              "ge": np.greater_equal, "isclose": np.isclose, "arctan2": np.arctan2}
_NP_UNARY = {"neg": np.negative, "abs": np.absolute, "log": np.log, "exp": np.exp, "floor": np.floor,
             "ceil": np.ceil, "sign": np.sign, "sqrt": np.sqrt, "square": np.square, "log10": np.log10,
             "sin": np.sin, "cos": np.cos, "tan": np.tan, "arcsin": np.arcsin, "arccos": np.arccos,
             "arctan": np.arctan, "sinh": np.sinh, "cosh": np.cosh, "tanh": np.tanh, "arcsinh": np.arcsinh,
             "arccosh": np.arccosh, "arctanh": np.arctanh}
_COMPARISONS = {"eq", "ne", "lt", "le", "gt", "ge", "isclose"}


def _numpy_result(op, dta, dtb=None):
    """numpy's own answer for the result dtype (and its TypeError for e.g. bool - bool)."""
    a = np.ones(1, dtype=dta)
    with np.errstate(all="ignore"):
        if dtb is None:
            return _NP_UNARY[op](a).dtype
        return _NP_BINARY[op](a, np.ones(1, dtype=dtb)).dtype


def _elementwise(op, a, b, n, out_dt, compute_dt, flag):
    out = _alloc(n, out_dt)
    oa = _operand(a)
    ob = _operand(b) if b is not None else oa
    lib = _lib.load()
    _lib.check(lib.pbh_elementwise(_lib.OPS[op], _PBH_DTYPE[_canonical(compute_dt)], _PBH_DTYPE[_canonical(out_dt)],
                                   oa, ob, out.data_ptr(), n, flag, device.stream()), f"transform {op}")
    return out


def _binary(op, a, b, n, flag=None):
    dta, dtb = _dtype_of(a), _dtype_of(b)
    res = _numpy_result(op, dta, dtb)
    if isinstance(a, _Broadcast) and isinstance(b, _Broadcast):
        with np.errstate(all="ignore"):
            v = _NP_BINARY[op](np.ones(1, dta) * a.value, np.ones(1, dtb) * b.value)
        if op == "pow" and np.issubdtype(res, np.integer) and b.value < 0:
            raise ValueError("Integers to negative integer powers are not allowed.")
        return _Broadcast(v[0], n, res)
    out_dt = _canonical(res)
    if op in _COMPARISONS or op in ("and", "or"):
        compute = _canonical(np.result_type(dta, dtb))
        if op in ("isclose", "and", "or"):
            compute = np.dtype(np.float64)
    else:
        compute = out_dt
    return _elementwise(op, a, b, n, out_dt, compute, flag)


def _unary(op, a, n, flag=None):
    dta = _dtype_of(a)
    res = _numpy_result(op, dta)
    if isinstance(a, _Broadcast):
        with np.errstate(all="ignore"):
            v = _NP_UNARY[op](np.ones(1, dta) * a.value)
        return _Broadcast(v[0], n, res)
    out_dt = _canonical(res)
    compute = out_dt
    if op not in ("neg", "abs", "sign", "square", "floor", "ceil") and out_dt != np.float64:
        compute = np.dtype(np.float64)
    return _elementwise(op, a, None, n, out_dt, compute, flag)


# =============================================================================
# COMPUTATIONAL GRAPH AND MODELING LANGUAGE
# =============================================================================
class _GraphPlan:
    __slots__ = ("G", "all_nodes", "isns", "order", "n_dist")

    def __init__(self, G, all_nodes, isns, order, n_dist):
        self.G, self.all_nodes, self.isns, self.order, self.n_dist = G, all_nodes, isns, order, n_dist


class Node(abc.ABC):
    """A node in the computational graph (modeling.py:335-680)."""

    id_iter = itertools.count()  # creation order = the ISN column order (modeling.py:525)

    def __init__(self):
        self._id = next(self.id_iter)
        self._correlations = []

    def __eq__(self, other):
        if not isinstance(other, Node):
            return NotImplemented
        return self._id == other._id

    def __hash__(self):
        return self._id

    # ---- samples: device vector + lazily materialised numpy view ----------------
    @property
    def samples_(self):
        d = self.__dict__
        if "_smp" not in d:
            raise AttributeError(f"'{type(self).__name__}' object has no attribute 'samples_'")
        dev = d["_smp"]
        if dev is None:
            return None
        if d.get("_host") is None:
            d["_host"] = dev.host() if isinstance(dev, _Broadcast) else device.to_host(dev)
        return d["_host"]

    @samples_.setter
    def samples_(self, value):
        self.__dict__["_smp"] = _to_device_samples(value)
        self.__dict__["_host"] = value if isinstance(value, np.ndarray) else None

    @samples_.deleter
    def samples_(self):
        if "_smp" not in self.__dict__:
            raise AttributeError("samples_")
        del self.__dict__["_smp"]
        self.__dict__.pop("_host", None)

    @property
    def samples_device(self):
        """The device tensor behind `samples_` (a scalar broadcast is materialised)."""
        dev = self.__dict__["_smp"]
        if isinstance(dev, _Broadcast):
            dev = _elementwise("cast", dev, None, dev.n, dev.dtype, dev.dtype, None)
        return dev

    def _set_device(self, dev):
        self.__dict__["_smp"] = dev
        self.__dict__["_host"] = None

    def _dev(self):
        return self.__dict__["_smp"]

    # ---- graph -------------------------------------------------------------------
    def copy(self):
        """Copy the node and the graph above it (modeling.py:353-404)."""
        new = {}

        def remap(item):
            return new[item._id] if isinstance(item, Node) else copy.deepcopy(item)

        for node in nx.topological_sort(self.to_graph()):
            dup = copy.copy(node)
            dup.__dict__ = dict(node.__dict__)
            dup.__dict__.pop("_plan_cache", None)  # it names the original's nodes
            new[dup._id] = dup
            dev = dup.__dict__.get("_smp")
            if dev is not None and not isinstance(dev, _Broadcast):
                dup.__dict__["_smp"] = dev.clone()
                dup.__dict__["_host"] = None
            dup._correlations = copy.deepcopy(dup._correlations)
            if isinstance(dup, (AbstractDistribution, ScalarFunctionTransform)) and hasattr(dup, "args"):
                dup.args = tuple(remap(a) for a in dup.args)
                dup.kwargs = {k: remap(v) for k, v in dup.kwargs.items()}
            elif isinstance(dup, (VariadicTransform, BinaryTransform)):
                dup.parents = tuple(remap(p) for p in dup.parents)
            elif isinstance(dup, UnaryTransform):
                dup.parent = remap(dup.parent)
            elif isinstance(dup, MarginalDistribution):
                dup.distr = remap(dup.distr)
            elif isinstance(dup, Constant):
                dup.value = remap(dup.value)
        return new[self._id]

    def nodes(self):
        """Yield self and all ancestors, depth first (modeling.py:406-423)."""
        stack = [self]
        while stack:
            node = stack.pop()
            yield node
            stack.extend(node.get_parents())

    def num_distribution_nodes(self):
        return self._plan().n_dist

    def _plan(self):
        """The graph analysis of an evaluation (networkx graph, topological order, ISNs), kept on
        the node between calls: the reference redoes it on every .sample() (modeling.py:499-538),
        ~1 ms of Python for cfg3's 33 nodes.  It is reused only while a walk over the ancestors
        finds the same node objects with the same correlation counts (a node's parents are fixed
        at construction; correlate() appends), so a changed graph is always analysed again."""
        fp = tuple((id(n), len(n._correlations)) for n in self.nodes())
        cached = self.__dict__.get("_plan_cache")
        if cached is not None and cached[0] == fp:
            return cached[1]
        G = self.to_graph()
        assert nx.is_directed_acyclic_graph(G)
        all_nodes = set(G.nodes) if G.number_of_nodes() else {self}
        plan = _GraphPlan(G, all_nodes, sorted({n for n in all_nodes if n._is_initial_sampling_node()},
                                               key=lambda n: n._id),
                          list(nx.topological_sort(G)),
                          sum(1 for node in all_nodes if isinstance(node, AbstractDistribution)))
        self.__dict__["_plan_cache"] = (fp, plan)
        return plan

    def to_graph(self):
        """networkx MultiDiGraph of the expression (modeling.py:663-680)."""
        nodes = list(self.nodes())
        if len(nodes) == 1:
            G = nx.MultiDiGraph()
            G.add_node(self)
            return G
        return nx.MultiDiGraph([(parent, node) for node in nodes for parent in node.get_parents()
                                if not node.is_leaf])

    def _is_initial_sampling_node(self):
        """A Distribution none of whose ancestors is a Distribution (modeling.py:616-626)."""
        if not isinstance(self, AbstractDistribution):
            return False
        return not any(isinstance(n, AbstractDistribution) for n in set(self.nodes()) - {self})

    def correlate(self, *variables, corr_mat):
        """Record a correlation between ancestor variables (modeling.py:628-661)."""
        assert corr_mat.ndim == 2
        assert corr_mat.shape[0] == corr_mat.shape[1]
        assert corr_mat.shape[0] == len(variables)
        assert len(variables) == len(set(variables))
        ancestors = set(self.nodes())
        for var in variables:
            if var not in ancestors:
                raise ValueError(f"{var} is not an ancestor of {self}")
        self._correlations.append((list(variables), np.copy(corr_mat)))
        return self

    # ---- sampling ----------------------------------------------------------------
    def sample(self, size=None, random_state=None, method=None, correlator="imanconover", gc_strategy=None,
               stream=None):
        """Sample this node and assign `.samples_` on every ancestor (modeling.py:431-493).

        The quantile matrix is generated on the GPU (see probabilit_amd.qmc) and never
        materialised for method="lhs" (generator fused into the inverse-CDF kernels).

        stream (extra, keyword): for method="lhs", "native" (default: the counter-based
        design) or "reference" (scipy's LatinHypercube(d, rng=random_state).random(size) bit
        for bit, so results equal the reference's on the same seed); None takes the module
        default (probabilit_amd.qmc.set_default_stream, env PBH_LHS_STREAM).  method=None,
        "sobol" and "halton" always reproduce the reference's streams."""
        size = 1 if size is None else size
        d = self.num_distribution_nodes()
        if method is not None and method.lower().strip() not in ("lhs", "halton", "sobol"):
            raise KeyError(method.lower().strip())
        source = qmc.make_source(method, size, d, random_state, stream=stream)
        return self._evaluate(source, correlator, gc_strategy, to_host=True)

    def sample_from_quantiles(self, quantiles, correlator="imanconover", gc_strategy=None):
        """Evaluate the graph on given quantiles, shape (samples, dimensions) (modeling.py:495-614)."""
        src = qmc.DeviceMatrixSource(quantiles)
        return self._evaluate(src, correlator, gc_strategy, to_host=True)

    def sample_device(self, size=None, random_state=None, method=None, correlator="imanconover",
                      gc_strategy=None, group=None, stream=None):
        """As sample(), but return the sink's device tensor (no D2H copy).

        group: a torch.distributed process group (one process per GPU).  With more than one
        rank the `size` rows are sharded: rank r evaluates every node on the rows
        [size r / R, size (r + 1) / R) and returns its rows of the sink; generators are
        counter-addressed by the global row, correlations run through the row-sharded
        Iman-Conover of probabilit_amd.distributed."""
        size = 1 if size is None else size
        source = qmc.make_source(method, size, self.num_distribution_nodes(), random_state, stream=stream)
        return self._evaluate(source, correlator, gc_strategy, to_host=False, group=group)

    def _evaluate(self, source, correlator, gc_strategy, to_host, group=None):
        plan = self._plan()
        G = plan.G
        n_dim = source.d
        assert n_dim == plan.n_dist
        world, rank = 1, 0
        if group is not None:
            import torch.distributed as tdist

            world, rank = tdist.get_world_size(group), tdist.get_rank(group)
        if world > 1:
            from .distributed import shard_bounds

            rb = shard_bounds(source.n, world)
            source.shard(rb[rank], rb[rank + 1] - rb[rank])
        size = source.rows  # the rows this process evaluates

        if isinstance(correlator, str):
            correlator = {"imanconover": ImanConover, "cholesky": Cholesky}[correlator.lower()]

        all_nodes = plan.all_nodes
        for node in all_nodes:
            if "_smp" in node.__dict__:
                del node.samples_

        gc = GarbageCollector(strategy=gc_strategy).set_sink(self)
        isns = plan.isns
        isn_set = set(isns)
        ev = _Evaluation(size, list(G.nodes))

        # correlations are a property of the graph: gather and validate them first so that
        # the correlated ISNs can be written straight into one (K, N) block (:542-568)
        correlations = []
        for node in all_nodes:
            correlations.extend(getattr(node, "_correlations", []))
        variable_sets = [set(v) for (v, _) in correlations]
        all_variables = sorted(functools.reduce(set.union, variable_sets, set()), key=lambda n: n._id)
        block, block_row = None, {}
        # Fast path: correlated ISNs drawn from the native LHS with plain-number parameters
        # are handed to Iman-Conover as generator descriptors; their uncorrelated samples are
        # overwritten by the correlator anyway (:582-583), so they are never materialised.
        all_set = set(all_variables)
        generated = (bool(correlations) and isinstance(source, qmc.LHSSource)
                     and isinstance(correlator, type) and issubclass(correlator, ImanConover)
                     and all_set <= isn_set
                     and all(type(v) is Distribution and v.distr in _FUSED_LHS and v.is_leaf
                             for v in all_variables))
        deferred = {}
        if correlations and all_set <= isn_set and not generated:
            block = device.empty((len(all_variables), size))
            block_row = {v: j for j, v in enumerate(all_variables)}

        # a graph of leaf draws, constants and float64 transforms runs as one kernel
        fused = not correlations and dag.try_evaluate(list(plan.order), isns, source, ev, gc)
        if not fused:
            # the ISNs' quantile columns in the reference's order (:529-538); native-LHS leaves with
            # plain-number parameters are then drawn together by one call (pbh_lhs_ppf_columns: their
            # inverse-CDF setups overlap), the rest one by one
            if correlations and block is not None and isinstance(source, qmc.ReferenceLHSSource) and world == 1:
                source.keep_strata = True  # the correlated leaves' ranks (step 1 of Iman-Conover)
            columns, col_index = {}, {}
            for node in isns:
                col_index[node] = source._next
                columns[node] = source.next_column()
            leaves = []
            if isinstance(source, qmc.LHSSource):
                leaves = [node for node in isns
                         if type(node) is Distribution and node.is_leaf and node.distr in _FUSED_LHS
                         and not (generated and node in all_set) and node not in block_row
                         and all(not isinstance(v, Node) and np.ndim(v) == 0
                                 for v in _parse_scipy_args(node.distr, node.args, node.kwargs))]
            if len(leaves) >= 2:
                leaves = [(node, node._params(size)) for node in leaves]
                cols = []
                for node, params in leaves:
                    _, seed, n_total, col, row0 = columns[node]
                    cols.append(_lib.ICColumn(seed, col, _lib.DIST_IDS[node.distr],
                                              (ctypes.c_double * 4)(*(params + [0.0] * (4 - len(params)))),
                                              len(params), ev.flag_ptr(node)))
                gblock = device.empty((len(leaves), size))
                arr = (_lib.ICColumn * len(cols))(*cols)
                _lib.check(_lib.load().pbh_lhs_ppf_columns(arr, len(cols), source.n, source.row0, size,
                                                           gblock.data_ptr(), size, device.stream()),
                           "pbh_lhs_ppf_columns")
                for j, (node, _) in enumerate(leaves):
                    node._set_device(gblock[j])
            grouped = {node for node, _ in leaves} if len(leaves) >= 2 else ()
            for node in isns:  # (:529-538)
                if node in grouped:
                    continue
                if not node.is_leaf:  # (a leaf has no ancestors to sample)
                    for anc in nx.topological_sort(G.subgraph(nx.ancestors(G, node))):
                        assert isinstance(anc, (Constant, Transform))
                        anc._set_device(anc._sample_device(ev))
                assert isinstance(node, AbstractDistribution)
                if generated and node in all_set:
                    deferred[node] = columns[node]
                    continue
                out = block[block_row[node]] if node in block_row else None
                node._set_device(node._sample_device(ev, columns[node], out=out))

            for variables, _ in correlations:  # (:548-551)
                for variable in variables:
                    if variable not in isn_set:
                        raise ValueError(f"Cannot correlate variable: {variable}")
            for vars1, vars2 in itertools.combinations(variable_sets, 2):  # (:554-558)
                common = vars1.intersection(vars2)
                if len(common) > 1:
                    raise ValueError(f"Correlations specified more than once: {common}")

            if correlations:  # (:571-583)
                var_to_int = {v: i for (i, v) in enumerate(all_variables)}
                indexed = [(tuple(var_to_int[v] for v in vs), cm) for (vs, cm) in correlations]
                C = nearest_correlation_matrix(build_corrmat(indexed))
                inst = correlator().set_target(C)
                if generated and world > 1:
                    from .distributed import LHSColumn, iman_conover_lhs

                    cols = []
                    for var in all_variables:
                        _, seed, n_total, col, _ = deferred[var]
                        cols.append(LHSColumn(seed, col, _lib.DIST_IDS[var.distr], [float(p) for p in var._params(size)]))
                    vflags = device.zeros(len(cols), "int32")
                    Y = iman_conover_lhs(cols, inst.P, source.n, group=group, flags=vflags)
                    for j, var in enumerate(all_variables):
                        ev.flags[ev.slot[var]] |= vflags[j]  # bitmask words: OR, never add
                        var._set_device(Y[j])
                elif generated:
                    cols = []
                    for var in all_variables:
                        _, seed, n_total, col, _ = deferred[var]
                        params = [float(p) for p in var._params(size)]
                        cols.append(_lib.ICColumn(seed, col, _lib.DIST_IDS[var.distr], (ctypes.c_double * 4)(*params),
                                                  len(params), ev.flag_ptr(var)))
                    Y = inst._transform_generated(cols, size)
                    for j, var in enumerate(all_variables):
                        var._set_device(Y[j])
                elif world > 1:
                    # any other correlator on row shards
                    from . import distributed as _dist

                    assert block is not None  # every correlated variable is an ISN (checked above)
                    K = len(all_variables)
                    if isinstance(inst, ImanConover):
                        # sharded: each column ranked on its owner, Gram all-reduced, no replica
                        inst._validate_X(np.lib.stride_tricks.as_strided(np.zeros(1), (source.n, K), (0, 0)))
                        Y = _dist.iman_conover_block(block, inst.P, source.n, group=group)
                    elif isinstance(inst, Cholesky):
                        # row-local given the global means and Gram matrix: two all-reduces
                        stats = _dist.block_stats(block, source.n, group=group)
                        Y = inst._transform_device(block, ev, stats=stats, n=source.n)
                    else:
                        # state no rank can share by construction (an unseeded PermutationCorrelator's
                        # rng, a user class): the correlator runs once, on rank 0, over the whole
                        # block gathered there, and every rank receives its rows
                        full = _dist.gather_to_root(block, source.n, group)
                        Yf = None
                        if rank == 0:
                            if isinstance(inst, PermutationCorrelator):
                                Yf = inst._transform_device(full, ev)
                            else:  # a user correlator class: the reference's (N, K) ndarray protocol
                                Yf = device.to_device(np.ascontiguousarray(np.asarray(inst(device.to_host(full).T),
                                                                                      dtype=np.float64).T))
                        del full
                        Y = _dist.scatter_from_root(Yf, K, source.n, group, like=block)
                    for j, var in enumerate(all_variables):
                        var._set_device(Y[j])
                elif isinstance(inst, ImanConover) and getattr(source, "strata", None) is not None:
                    # leaves with plain-number parameters: their ranks are their LHS strata
                    # (checked on the device; a column that fails the check is sorted)
                    strata = [source.strata_of(col_index[v])
                              if type(v) is Distribution and v.is_leaf
                              and all(not isinstance(p, Node) and np.ndim(p) == 0
                                      for p in _parse_scipy_args(v.distr, v.args, v.kwargs)) else None
                              for v in all_variables]
                    Y = inst._transform_device(block, ev, strata=strata)
                    for j, var in enumerate(all_variables):
                        var._set_device(Y[j])
                elif isinstance(inst, (ImanConover, Cholesky, PermutationCorrelator)):
                    Y = inst._transform_device(block, ev)
                    for j, var in enumerate(all_variables):
                        var._set_device(Y[j])
                else:  # a user correlator class: the reference's (N, K) ndarray protocol
                    X = np.vstack([v.samples_ for v in all_variables]).T
                    Yh = inst(X)
                    for var, col in zip(all_variables, Yh.T):
                        var.samples_ = np.copy(col)

            if getattr(source, "strata", None) is not None:
                source.strata = None  # read only by the correlators above: d x n int32 freed now
            # the per-node loop, or all of it as one fused kernel (probabilit_amd.dag)
            order = list(plan.order)
            if correlations and dag.try_evaluate(order, isns, source, ev, gc):
                order = []
            for node in order:  # (:586-612)
                if "_smp" in node.__dict__:
                    pass
                elif isinstance(node, Constant):
                    node._set_device(node._sample_device(ev))
                elif isinstance(node, AbstractDistribution):
                    node._set_device(node._sample_device(ev, source.next_column()))
                elif isinstance(node, Transform):
                    node._set_device(node._sample_device(ev))
                else:
                    raise TypeError("Node must be Constant, AbstractDistribution or Transform.")
                gc.decrement_and_delete(node)

        # fused non-finite check (:600-606): first flagged node in topological order raises
        if world > 1:  # every rank raises the same error (flag words OR-combined, bits unchanged)
            from .distributed import _all_reduce_flags

            _all_reduce_flags(ev.flags, group, world)
        flags = device.to_host(ev.flags)
        if flags.any():
            for node in nx.topological_sort(G):
                if flags[ev.slot[node]] & 4:  # DiscreteDistribution: q past the last cumulative
                    m = len(node.probabilities)
                    raise IndexError(f"index {m} is out of bounds for axis 0 with size {m}")
                if flags[ev.slot[node]] & 2:  # numpy's integer power check
                    raise ValueError("Integers to negative integer powers are not allowed.")
                if flags[ev.slot[node]]:
                    shown = node.samples_ if "_smp" in node.__dict__ else "(garbage collected)"
                    raise ValueError(f"Sampling this node gave non-finite values: {node}\n{shown}")

        if not to_host:
            return None if self._dev() is None else self.samples_device
        # the reference leaves numpy samples_ on every node (modeling.py:582-583, 598, 614): hand
        # them all back in one pipelined batch (device.to_host_many) rather than one by one
        pending = [nd for nd in set(self.nodes()) if "_smp" in nd.__dict__ and nd.__dict__.get("_host") is None
                   and nd.__dict__["_smp"] is not None and not isinstance(nd.__dict__["_smp"], _Broadcast)]
        for nd, host in zip(pending, device.to_host_many([nd.__dict__["_smp"] for nd in pending])):
            nd.__dict__["_host"] = host
        return self.samples_


class OverloadMixin:
    """Arithmetic and comparison operators build Transform nodes (modeling.py:683-748)."""

    def __add__(self, other): return Add(self, other)
    def __radd__(self, other): return Add(self, other)
    def __mul__(self, other): return Multiply(self, other)
    def __rmul__(self, other): return Multiply(self, other)
    def __floordiv__(self, other): return FloorDivide(self, other)
    def __rfloordiv__(self, other): return FloorDivide(other, self)
    def __truediv__(self, other): return Divide(self, other)
    def __rtruediv__(self, other): return Divide(other, self)
    def __mod__(self, other): return Mod(self, other)
    def __rmod__(self, other): return Mod(other, self)
    def __sub__(self, other): return Subtract(self, other)
    def __rsub__(self, other): return Subtract(other, self)
    def __pow__(self, other): return Power(self, other)
    def __rpow__(self, other): return Power(other, self)
    def __neg__(self): return Negate(self)
    def __abs__(self): return Abs(self)
    def __lt__(self, other): return LessThan(self, other)
    def __le__(self, other): return LessThanOrEqual(self, other)
    def __gt__(self, other): return GreaterThan(self, other)
    def __ge__(self, other): return GreaterThanOrEqual(self, other)


class Constant(Node, OverloadMixin):
    """A number; sampled as a lazily broadcast scalar (modeling.py:751-769)."""

    is_leaf = True

    def __init__(self, value):
        self.value = value.value if isinstance(value, Constant) else value
        super().__init__()

    def _sample(self, size=None):
        if size is None:
            return self.value
        return np.ones(size, dtype=type(self.value)) * self.value

    def _sample_device(self, ev):
        return _Broadcast(self.value, ev.size)

    def get_parents(self):
        yield from []

    def __repr__(self):
        return f"{type(self).__name__}({self.value})"


class AbstractDistribution(Node, OverloadMixin, abc.ABC):
    pass


# scipy.stats parameter layout of the distributions with native kernels: shape names,
# then loc (and scale for continuous ones) -- scipy's rv_generic._parse_args.
_DIST_SHAPES = {"norm": (), "uniform": (), "expon": (), "lognorm": ("s",), "triang": ("c",),
                "gamma": ("a",), "poisson": ("mu",), "beta": ("a", "b"), "truncnorm": ("a", "b"),
                "binom": ("n", "p"), "bernoulli": ("p",), "weibull_min": ("c",), "weibull_max": ("c",),
                "logistic": (), "cauchy": (), "laplace": (), "gumbel_r": (), "gumbel_l": (), "pareto": ("b",),
                "loguniform": ("a", "b"), "reciprocal": ("a", "b"), "rayleigh": (), "lomax": ("c",),
                "genextreme": ("c",), "gompertz": ("c",), "chi2": ("df",), "erlang": ("a",),
                "halfcauchy": (), "halflogistic": (), "halfnorm": (), "arcsine": (), "hypsecant": (),
                "powerlaw": ("a",), "genpareto": ("c",), "fisk": ("c",), "burr": ("c", "d"),
                "burr12": ("c", "d"), "exponweib": ("a", "c"), "exponpow": ("b",), "bradford": ("c",),
                "anglit": (), "levy": (), "levy_l": (), "gibrat": (), "invweibull": ("c",),
                "loglaplace": ("c",), "truncexpon": ("b",), "chi": ("df",), "maxwell": (), "nakagami": ("nu",),
                "dweibull": ("c",), "kappa3": ("a",), "genhalflogistic": ("c",), "alpha": ("a",),
                "fatiguelife": ("c",), "genlogistic": ("c",), "trapezoid": ("c", "d"),
                "geom": ("p",), "randint": ("low", "high"), "nbinom": ("n", "p"), "invgamma": ("a",), "t": ("df",),
                # round 6
                "trapz": ("c", "d"), "johnsonsu": ("a", "b"), "johnsonsb": ("a", "b"), "powernorm": ("c",),
                "laplace_asymmetric": ("kappa",), "mielke": ("k", "s"), "truncpareto": ("b", "c"),
                "tukeylambda": ("lam",), "gengamma": ("a", "c"), "loggamma": ("c",), "dgamma": ("a",),
                "f": ("dfn", "dfd"), "rdist": ("c",), "semicircular": (), "betaprime": ("a", "b"),
                "dlaplace": ("a",), "planck": ("lambda_",), "boltzmann": ("lambda_", "N"),
                "pearson3": ("skew",), "gennorm": ("beta",), "halfgennorm": ("beta",), "wrapcauchy": ("c",),
                "skewcauchy": ("a",), "moyal": (), "kappa4": ("h", "k"), "crystalball": ("beta", "m"),
                "powerlognorm": ("c", "s"), "jf_skew_t": ("a", "b"), "foldcauchy": ("c",), "foldnorm": ("c",),
                "cosine": (), "invgauss": ("mu",), "wald": (), "betabinom": ("n", "a", "b"), "hypergeom": ("M", "n", "N"),
                "skewnorm": ("a",), "recipinvgauss": ("mu",), "exponnorm": ("K",), "argus": ("chi",), "kstwobign": (),
                "nhypergeom": ("M", "n", "r"), "yulesimon": ("alpha",),
                "zipfian": ("a", "n"), "rel_breitwigner": ("rho",)}
_DISCRETE = {"poisson", "binom", "bernoulli", "geom", "randint", "nbinom", "dlaplace", "planck", "boltzmann", "betabinom",
             "hypergeom", "nhypergeom", "yulesimon", "zipfian"}
# distributions with a fused native-LHS + inverse-CDF kernel and a stratum-ordered generator, so
# that Iman-Conover takes them as generated columns (pbh_ppf.hip k_lhs_sorted_ppf / k_place_gen;
# the extended set pbh_ppf_ext.hip k_ext_sorted / k_ext_place): every distribution with a kernel
_FUSED_LHS = set(_DIST_SHAPES)


def _parse_scipy_args(name, args, kwargs):
    shapes = _DIST_SHAPES[name]
    names = list(shapes) + (["loc"] if name in _DISCRETE else ["loc", "scale"])
    defaults = {"loc": 0.0, "scale": 1.0}
    if len(args) > len(names):
        raise TypeError(f"_parse_args() takes from {len(shapes)} to {len(names)} positional arguments but "
                        f"{len(args)} were given")
    vals = dict(zip(names, args))
    for k, v in kwargs.items():
        if k not in names:
            raise TypeError(f"_parse_args() got an unexpected keyword argument '{k}'")
        if k in vals:
            raise TypeError(f"_parse_args() got multiple values for argument '{k}'")
        vals[k] = v
    missing = [s for s in shapes if s not in vals]
    if missing:
        raise TypeError(f"_parse_args() missing {len(missing)} required positional argument: '{missing[0]}'")
    return [vals.get(nm, defaults.get(nm)) for nm in names]


class Distribution(AbstractDistribution):
    """A scipy.stats distribution sampled by inverse CDF on the GPU (modeling.py:776-822)."""

    def __init__(self, distr, *args, **kwargs):
        self.distr = distr
        self.args = args
        self.kwargs = kwargs
        super().__init__()

    def __repr__(self):
        args = ", ".join(repr(arg) for arg in self.args)
        kwargs = ", ".join(f"{k}={repr(v)}" for (k, v) in self.kwargs.items())
        out = f'{type(self).__name__}("{self.distr}"'
        if args:
            out += f", {args}"
        if kwargs:
            out += f", {kwargs}"
        return out + ")"

    def _params(self, n):
        name = self.distr
        getattr(scipy.stats, name)  # AttributeError for unknown names, as getattr(stats, ...) at :805
        if name not in _DIST_SHAPES:
            raise NotImplementedError(f"Distribution('{name}') has no native inverse-CDF kernel yet; supported: "
                                      f"{sorted(_DIST_SHAPES)}")

        def resolve(v):
            if isinstance(v, Node):
                return _as_float_vector(v._dev(), n)
            a = np.asarray(v, dtype=np.float64)
            if a.ndim == 0:
                return float(a)
            if a.shape != (n,):
                raise NotImplementedError(f"array-valued parameter of shape {a.shape} for size {n}")
            return device.to_device(a)

        vals = _parse_scipy_args(name, self.args, self.kwargs)
        if name == "erlang" and not isinstance(vals[0], Node) and not np.all(np.floor(vals[0]) == vals[0]):
            # scipy's erlang_gen._argcheck warns (and samples anyway)
            warnings.warn("The shape parameter of the erlang distribution has been given a non-integer value "
                          f"{np.asarray(vals[0])!r}.", RuntimeWarning, stacklevel=4)
        return [resolve(v) for v in vals]

    def _sample_device(self, ev, column, out=None):
        n = ev.size
        params = self._params(n)
        keep = [p for p in params if not isinstance(p, float)]  # keep vectors alive over the launch
        arr = (_lib.Param * len(params))(*[_lib.Param(None, p) if isinstance(p, float) else _lib.Param(p.data_ptr(), 0.0)
                                            for p in params])
        out = device.empty(n) if out is None else out
        lib = _lib.load()
        dist = _lib.DIST_IDS[self.distr]
        if column[0] == "lhs":
            _, seed, n_total, col, row0 = column
            _lib.check(lib.pbh_lhs_ppf(seed, n_total, row0, n, col, dist, arr, len(params), out.data_ptr(),
                                       ev.flag_ptr(self), device.stream()), f"{self}")
        elif column[0] == "sobol" and dist < _lib.DIST_IDS["beta"]:  # generator fused into the ppf kernel
            _, src, col = column
            sv = np.ascontiguousarray(src.sv, dtype=np.uint32)
            sh = np.ascontiguousarray(src.shift, dtype=np.uint32)
            _lib.check(lib.pbh_sobol_ppf(_lib.np_ptr(sv), _lib.np_ptr(sh), src.d, src.bits, src.row0, n, col, dist, arr,
                                         len(params), out.data_ptr(), ev.flag_ptr(self), device.stream()), f"{self}")
        else:
            if column[0] == "sobol":
                column = ("vector", column[1].materialize(column[2]), 1)
            _, q, stride = column
            _lib.check(lib.pbh_ppf(dist, q.data_ptr(), stride, n, arr, len(params), out.data_ptr(),
                                   ev.flag_ptr(self), device.stream()), f"{self}")
        del keep
        return out

    def get_parents(self):
        for arg in self.args + tuple(self.kwargs.values()):
            if isinstance(arg, Node):
                yield arg

    @property
    def is_leaf(self):
        return list(self.get_parents()) == []


def _into(res, out):
    """Write a node's samples into a preallocated float64 row (the correlated block) if given."""
    if out is None:
        return res
    out.copy_(res)
    return out


_QUANTILE_METHODS = {"linear": 0, "lower": 1, "higher": 2, "nearest": 3, "midpoint": 4}


class _TableDistribution(AbstractDistribution):
    """Leaf distribution given by a host table; sampled on the device by pbh_table_ppf.  The
    table (at most a few thousand entries, independent of the sample size) is prepared on the
    host once and cached on the device."""

    is_leaf = True

    def get_parents(self):
        yield from []

    @staticmethod
    def _quantile_column(column, n):
        """(device q vector, stride) of this node's quantile column; a fused native-LHS column
        is materialised (pbh_fill_lhs)."""
        if column[0] == "lhs":
            _, seed, n_total, col, row0 = column
            q = device.empty(n)
            _lib.check(_lib.load().pbh_fill_lhs(seed, n_total, row0, n, col, 1, q.data_ptr(), max(n, 1),
                                                device.stream()), "pbh_fill_lhs")
            return q, 1
        if column[0] == "sobol":
            return column[1].materialize(column[2]), 1
        _, q, stride = column
        return q, stride

    def _sample(self, q):
        """The reference's `_sample(q)` (inverse CDF of explicit quantiles), on the device."""
        q = np.asarray(q, dtype=np.float64)
        qd = device.to_device(np.ascontiguousarray(q.ravel()))
        ev = _Evaluation(qd.shape[0], [self])
        res = device.to_host(self._sample_device(ev, ("vector", qd, 1)))
        flags = device.to_host(ev.flags)
        if flags[0] & 4:
            m = len(self.probabilities)
            raise IndexError(f"index {m} is out of bounds for axis 0 with size {m}")
        labels = self.__dict__.get("_labels")
        res = res if labels is None else labels[res]
        return res.reshape(q.shape)

    def _tables(self):
        cache = self.__dict__.get("_dev_tables")
        if cache is None:
            cache = self.__dict__["_dev_tables"] = self._build_tables()
        return cache

    def _launch(self, ev, column, kind, t0, t1, m, method, out_dt):
        n = ev.size
        q, stride = self._quantile_column(column, n)
        out = device.empty(n, out_dt)
        _lib.check(_lib.load().pbh_table_ppf(kind, q.data_ptr(), stride, n, t0.data_ptr(),
                                             None if t1 is None else t1.data_ptr(), m, method,
                                             _PBH_DTYPE[np.dtype(out_dt)], out.data_ptr(), ev.flag_ptr(self),
                                             device.stream()), f"{self}")
        return out


class EmpiricalDistribution(_TableDistribution):
    """np.quantile of data (modeling.py:825-844) on the device (pbh_table_ppf QUANTILE).
    Supported np.quantile keywords: method in linear (default) / lower / higher / nearest /
    midpoint; the data are flattened as np.quantile does with axis=None."""

    def __init__(self, data, **kwargs):
        self.data = np.array(data)
        self.kwargs = kwargs
        super().__init__()

    def __repr__(self):
        return f"{type(self).__name__}()"

    def _method(self):
        extra = set(self.kwargs) - {"method"}
        if extra:
            raise NotImplementedError(f"EmpiricalDistribution: np.quantile keywords {sorted(extra)} have no device path")
        method = self.kwargs.get("method", "linear")
        if method not in _QUANTILE_METHODS:
            raise NotImplementedError(f"np.quantile method={method!r} has no device path; "
                                      f"supported: {sorted(_QUANTILE_METHODS)}")
        return method

    def _build_tables(self):
        data = np.sort(np.asarray(self.data).ravel()).astype(np.float64)
        if data.size == 0:
            raise IndexError("index -1 is out of bounds for axis 0 with size 0")
        return (device.to_device(data),)

    def _sample_device(self, ev, column, out=None):
        return _into(self._sample_table(ev, column), out)

    def _sample_table(self, ev, column):
        method = self._method()
        (t0,) = self._tables()
        res = self._launch(ev, column, _lib.TABLE_QUANTILE, t0, None, t0.shape[0], _QUANTILE_METHODS[method],
                           "float64")
        if method in ("lower", "higher", "nearest") and np.issubdtype(self.data.dtype, np.integer):
            res = _elementwise("cast", res, None, ev.size, np.dtype(np.int64), np.dtype(np.int64), None)
        return res


class CumulativeDistribution(_TableDistribution):
    """Piecewise-linear inverse CDF (modeling.py:847-882): np.interp on the device."""

    def __init__(self, quantiles, cumulatives):
        self.q = np.array(quantiles)
        self.cumulatives = np.array(cumulatives)
        if not np.all(np.diff(self.q) > 0):
            raise ValueError("The quantiles must be strictly increasing.")
        if not np.all(np.diff(self.cumulatives) > 0):
            raise ValueError("The cumulatives must be strictly increasing.")
        if not (np.isclose(np.min(self.q), 0) and np.isclose(np.max(self.q), 1)):
            raise ValueError("Lowest quantile must be 0 and highest must be 1.")
        super().__init__()

    def __repr__(self):
        return f"{type(self).__name__}(quantiles={repr(self.q)}, cumulatives={repr(self.cumulatives)})"

    def _build_tables(self):
        return (device.to_device(np.asarray(self.q, dtype=np.float64)),
                device.to_device(np.asarray(self.cumulatives, dtype=np.float64)))

    def _sample_device(self, ev, column, out=None):
        return _into(self._sample_table(ev, column), out)

    def _sample_table(self, ev, column):
        xp, fp = self._tables()
        return self._launch(ev, column, _lib.TABLE_INTERP, xp, fp, xp.shape[0], 0, "float64")


class DiscreteDistribution(_TableDistribution):
    """Categorical values with probabilities (modeling.py:885-927):
    values[searchsorted(cumsum(p), q, side='right')] on the device.  Numeric values are
    gathered on the device; other values (e.g. strings) are sampled as indices on the device
    and mapped to the labels when `.samples_` is read (they cannot enter arithmetic)."""

    def __init__(self, values, probabilities=None):
        self.values = np.array(values)
        if probabilities is None:
            self.probabilities = np.ones(len(self.values), dtype=float)
            self.probabilities = self.probabilities / np.sum(self.probabilities)
        else:
            self.probabilities = np.array(probabilities)
        if not len(self.values) == len(self.probabilities):
            raise ValueError(f"Length mismatch: {len(self.values)=}  {len(self.probabilities)=}")
        if not np.isclose(np.sum(self.probabilities), 1.0):
            raise ValueError(f"Probabilities must sum to 1. {sum(self.probabilities)=}")
        if np.any(self.probabilities < 0):
            raise ValueError("Probabilities are not non-negative.")
        super().__init__()

    def __repr__(self):
        return f"{type(self).__name__}(values={repr(self.values)}, probabilities={repr(self.probabilities)})"

    def _kind(self):
        dt = self.values.dtype
        if dt == np.bool_ or np.issubdtype(dt, np.integer):
            return "int64"
        if np.issubdtype(dt, np.floating):
            return "float64"
        return None  # labels

    def _build_tables(self):
        cum = np.cumsum(self.probabilities).astype(np.float64)  # the reference's host cumsum, bit for bit
        kind = self._kind()
        vals = None if kind is None else device.to_device(self.values.astype(kind))
        return device.to_device(cum), vals

    def _sample_device(self, ev, column, out=None):
        return _into(self._sample_table(ev, column), out)

    def _sample_table(self, ev, column):
        cum, vals = self._tables()
        kind = self._kind() or "int64"
        res = self._launch(ev, column, _lib.TABLE_SEARCH, cum, vals, cum.shape[0], 0, kind)
        self.__dict__["_labels"] = self.values if self._kind() is None else None
        if self.values.dtype == np.bool_:
            res = _elementwise("cast", res, None, ev.size, np.dtype(bool), np.dtype(np.int64), None)
        return res

    def _samples_get(self):
        v = Node.samples_.fget(self)
        labels = self.__dict__.get("_labels")
        return v if labels is None or v is None else labels[v]

    samples_ = property(_samples_get, Node.samples_.fset, Node.samples_.fdel)

    def _dev(self):
        if self.__dict__.get("_labels") is not None:
            raise TypeError(f"{self!r}: non-numeric values cannot enter device arithmetic")
        return super()._dev()


# =============================================================================
# Transforms (modeling.py:933-1169)
# =============================================================================
class Transform(Node, OverloadMixin, abc.ABC):
    is_leaf = False

    def __repr__(self):
        return f"{type(self).__name__}({', '.join(repr(p) for p in self.get_parents())})"


class VariadicTransform(Transform):
    """functools.reduce(op, parents' samples) (modeling.py:943-959)."""

    op_name = None

    def __init__(self, *args):
        self.parents = tuple(python_to_prob(arg) for arg in args)
        super().__init__()

    def _sample_device(self, ev):
        n = ev.size
        acc = self.parents[0]._dev()
        for p in self.parents[1:]:
            acc = _binary(self.op_name, acc, p._dev(), n, ev.flag_ptr(self))
        return acc

    def get_parents(self):
        yield from self.parents


class Avg(VariadicTransform):
    """np.average(np.vstack(samples), axis=0) (modeling.py:986-990)."""

    def _sample_device(self, ev):
        n = ev.size
        f64 = np.dtype(np.float64)
        vecs = [_as_float_vector(p._dev(), n) for p in self.parents]
        vecs = [_elementwise("cast", _Broadcast(v, n), None, n, f64, f64, None) if isinstance(v, float) else v
                for v in vecs]
        out = device.empty(n)
        lib = _lib.load()
        ptrs = (ctypes.c_void_p * len(vecs))(*[v.data_ptr() for v in vecs])
        _lib.check(lib.pbh_average(ptrs, len(vecs), n, out.data_ptr(), ev.flag_ptr(self), device.stream()), "Avg")
        return out


class NoOp(VariadicTransform):
    """Sample all ancestors, produce nothing (modeling.py:993-997)."""

    def _sample_device(self, ev):
        return None


class BinaryTransform(Transform):
    """op(left, right) (modeling.py:1000-1012)."""

    op_name = None

    def __init__(self, *args):
        self.parents = tuple(python_to_prob(arg) for arg in args)
        super().__init__()

    def _sample_device(self, ev):
        a, b = (p._dev() for p in self.parents)
        return _binary(self.op_name, a, b, ev.size, ev.flag_ptr(self))

    def get_parents(self):
        yield from self.parents


class UnaryTransform(Transform):
    """op(parent) (modeling.py:1063-1075)."""

    op_name = None

    def __init__(self, arg):
        self.parent = python_to_prob(arg)
        super().__init__()

    def _sample_device(self, ev):
        return _unary(self.op_name, self.parent._dev(), ev.size, ev.flag_ptr(self))

    def get_parents(self):
        yield self.parent


def _define(base, table):
    for name, op in table.items():
        globals()[name] = type(name, (base,), {"op_name": op, "__module__": __name__})
        __all__.append(name)


_define(VariadicTransform, {"Add": "add", "Multiply": "mul", "Max": "max", "Min": "min", "All": "and",
                            "Any": "or"})
_define(BinaryTransform, {"FloorDivide": "floordiv", "Mod": "mod", "Divide": "truediv", "Power": "pow",
                          "Subtract": "sub", "Equal": "eq", "NotEqual": "ne", "LessThan": "lt",
                          "LessThanOrEqual": "le", "GreaterThan": "gt", "GreaterThanOrEqual": "ge",
                          "IsClose": "isclose", "Arctan2": "arctan2"})
_define(UnaryTransform, {"Negate": "neg", "Abs": "abs", "Log": "log", "Exp": "exp", "Floor": "floor",
                         "Ceil": "ceil", "Sign": "sign", "Sqrt": "sqrt", "Square": "square", "Log10": "log10",
                         "Sin": "sin", "Cos": "cos", "Tan": "tan", "Arcsin": "arcsin", "Arccos": "arccos",
                         "Arctan": "arctan", "Sinh": "sinh", "Cosh": "cosh", "Tanh": "tanh", "Arcsinh": "arcsinh",
                         "Arccosh": "arccosh", "Arctanh": "arctanh"})


class ScalarFunctionTransform(Transform):
    """A Python function applied sample by sample (modeling.py:1172-1201).  Inherently a
    scalar host loop: out of scope for the device path."""

    def __init__(self, func, args, kwargs):
        self.func = func
        self.args = args
        self.kwargs = kwargs
        super().__init__()

    def _sample_device(self, ev):
        raise NotImplementedError("scalar_transform runs a Python function per sample; it has no device path")

    def get_parents(self):
        for arg in self.args + tuple(self.kwargs.values()):
            if isinstance(arg, Node):
                yield arg


def scalar_transform(func):
    @functools.wraps(func)
    def transformed_function(*args, **kwargs):
        return ScalarFunctionTransform(func, args, kwargs)

    return transformed_function


class MarginalDistribution(Transform):
    """Slice of a multivariate distribution (modeling.py:1215-1243); pseudo-random .rvs only
    in the reference, so no inverse-CDF device path."""

    is_leaf = False

    def __init__(self, distr, d):
        self.distr = distr
        self.d = d
        super().__init__()

    def _sample_device(self, ev):
        raise NotImplementedError("multivariate distributions have no device path (SURVEY.md §2 #2)")

    def get_parents(self):
        yield self.distr

    def __repr__(self):
        return f"{type(self).__name__}({self.distr}, d={self.d})"


def MultivariateDistribution(distr, *args, **kwargs):
    """Marginals of a multivariate scipy distribution (modeling.py:1246-1264)."""
    dist = Distribution(distr, *args, **kwargs)
    frozen = getattr(scipy.stats, distr)(*args, **kwargs)
    d = len(np.atleast_1d(frozen.rvs(size=1, random_state=0)).squeeze())
    yield from (MarginalDistribution(dist, d=i) for i in range(d))

