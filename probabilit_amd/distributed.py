"""Row-sharded multi-GPU Iman-Conover over natively generated LHS columns.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Rank r of R owns
the rows [N r / R, N (r + 1) / R) of every column and the columns [K o / R, K (o + 1) / R)
for step 4.  The reference's single-process ImanConover.__call__ (correlation.py:368-425)
is split where its data dependencies cross rows:

    step 1  scores of the local rows, from the LHS permutation (no sort).  Discrete
            columns need the run heads of the sorted column: every rank extracts the heads
            of its own strata, one all-gather of the (short) head lists.
    step 2  column sums, then the centered Gram matrix of the local rows; each summed over
            ranks by an all-reduce (K and K x K doubles), then E = corrcoef and
            L = cholesky(E) on every rank's host (identical inputs -> identical L).
    step 3  CS = S L^-T P^T on the local rows.
    step 4  all-to-all of CS (row shards -> column owners), each owner ranks its full
            columns against their sorted values (generated locally), all-to-all of Y back
            to row shards.

The returned block is this rank's rows of every correlated column, (K, rows) on its GPU.
The compute of every phase goes through a `phases` object: `HipPhases` (the C-ABI of
libprobabilit_hip) in production; tests substitute a CPU implementation to exercise the
exchange logic under the gloo backend on machines without a GPU.
"""

import ctypes

import numpy as np

from . import _lib, device


def shard_bounds(n, world):
    """Row (and stratum) shard boundaries: rank r owns [b[r], b[r + 1])."""
    return [(n * r) // world for r in range(world + 1)]


class LHSColumn:
    """A generated column: stratum-addressable native LHS draw pushed through `dist`."""

    def __init__(self, seed, lhs_col, dist, params):
        self.seed = int(seed)
        self.lhs_col = int(lhs_col)
        self.dist = int(dist)
        self.params = [float(p) for p in params]


class HipPhases:
    """The Iman-Conover phases of include/probabilit_hip.h on this process's GPU."""

    def __init__(self):
        self.lib = _lib.load()
        self.dev = device.device()

    # -- allocation helpers -------------------------------------------------------------
    def empty(self, shape, dtype="float64"):
        return device.empty(shape, dtype)

    def _ws(self, nbytes):
        return device.empty(max(int(nbytes), 256), "uint8")

    # -- step 1 ---------------------------------------------------------------------------
    def sorted_segment(self, col, n, t0, nt, flag):
        out = device.empty(max(nt, 1))
        prm = (ctypes.c_double * 3)(*col.params)
        _lib.check(self.lib.pbh_lhs_sorted_ppf(col.seed, n, t0, nt, col.lhs_col, col.dist, prm, len(col.params),
                                               out.data_ptr(), flag.data_ptr(), device.stream()),
                   "pbh_lhs_sorted_ppf")
        return out[:nt]

    def sorted_check(self, x):
        ws = self._ws(256)
        ties, inv = ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.pbh_sorted_check(x.data_ptr(), x.shape[0], ctypes.byref(ties), ctypes.byref(inv),
                                             ws.data_ptr(), device.stream()), "pbh_sorted_check")
        return ties.value, inv.value

    def run_heads(self, x, t0, first_is_prev):
        m = x.shape[0]
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_run_heads_workspace_size(m, ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        heads = device.empty(max(m, 1), "int32")
        count = ctypes.c_int64()
        _lib.check(self.lib.pbh_run_heads(x.data_ptr(), m, t0, int(first_is_prev), heads.data_ptr(),
                                          ctypes.byref(count), ws.data_ptr(), nbytes.value, device.stream()),
                   "pbh_run_heads")
        return heads[:count.value]

    def scores(self, col, n, row0, nrows, heads, out):
        hp = heads.data_ptr() if heads is not None else None
        nh = heads.shape[0] if heads is not None else 0
        _lib.check(self.lib.pbh_lhs_scores(col.seed, n, col.lhs_col, row0, nrows, hp, nh, out.data_ptr(),
                                           device.stream()), "pbh_lhs_scores")

    # -- step 2 ---------------------------------------------------------------------------
    def _gram_ws(self, k):
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_gram_workspace_size(k, ctypes.byref(nbytes)))
        return self._ws(nbytes.value), nbytes.value

    def column_sums(self, S):
        k, n = S.shape
        out = device.zeros(k)
        if n:
            ws, nb = self._gram_ws(k)
            _lib.check(self.lib.pbh_column_sums(S.data_ptr(), n, k, S.stride(0), out.data_ptr(), ws.data_ptr(), nb,
                                                device.stream()), "pbh_column_sums")
        return out

    def centered_gram(self, S, means):
        k, n = S.shape
        out = device.zeros((k, k))
        if n:
            ws, nb = self._gram_ws(k)
            _lib.check(self.lib.pbh_centered_gram(S.data_ptr(), n, k, S.stride(0), means.data_ptr(), out.data_ptr(),
                                                  ws.data_ptr(), nb, device.stream()), "pbh_centered_gram")
        return out

    def factor(self, gram_host, n):
        k = gram_host.shape[0]
        g = np.ascontiguousarray(gram_host, dtype=np.float64)
        E = np.zeros((k, k))
        L = np.zeros((k, k))
        _lib.check(self.lib.pbh_ic_factor(g.ctypes.data, n, k, E.ctypes.data, L.ctypes.data), "pbh_ic_factor")
        return E, L

    # -- step 3 ---------------------------------------------------------------------------
    def apply(self, S, L, P):
        k, n = S.shape
        ws = self._ws((2 * k * k + k) * 8)
        Lh = np.ascontiguousarray(L, dtype=np.float64)
        Ph = np.ascontiguousarray(P, dtype=np.float64)
        _lib.check(self.lib.pbh_ic_apply(S.data_ptr(), n, k, S.stride(0), Lh.ctypes.data, Ph.ctypes.data,
                                         ws.data_ptr(), (2 * k * k + k) * 8, device.stream()), "pbh_ic_apply")

    # -- step 4 ---------------------------------------------------------------------------
    def reorder(self, cs, sorted_src, out):
        n = cs.shape[0]
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_ic_reorder_workspace_size(n, ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        _lib.check(self.lib.pbh_ic_reorder(cs.data_ptr(), n, sorted_src.data_ptr(), out.data_ptr(), 1, None,
                                           ws.data_ptr(), nbytes.value, device.stream()), "pbh_ic_reorder")


def _staged(group):
    """gloo moves host memory only: device tensors are staged through the host for it
    (used when several ranks share one GPU, e.g. in tests); RCCL/NCCL moves them in place."""
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def _all_gather_varlen(t, group, world):
    """Concatenation over ranks (in rank order) of 1-D tensors of different lengths."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return t
    dev = t.device
    if _staged(group):
        t = t.cpu()
    size = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(size) for _ in range(world)]
    dist.all_gather(sizes, size, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(max(sizes), 1)
    padded = torch.zeros(m, dtype=t.dtype, device=t.device)
    padded[:t.shape[0]] = t
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)]).to(dev)


def _all_reduce(t, group, world, op="sum"):
    import torch.distributed as dist

    if world > 1:
        red = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
        if _staged(group) and t.device.type != "cpu":
            h = t.cpu()
            dist.all_reduce(h, op=red, group=group)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=red, group=group)
    return t


def _all_reduce_flags(t, group, world, bits=3):
    """Combine per-node non-finite flag words (bitmasks: bit 0 non-finite value, bit 1 the
    integer-power error, bit 2 a DiscreteDistribution index past its table) across ranks
    without changing their bits: each bit plane is all-reduced with MAX (a bitwise OR;
    torch.distributed has no OR that RCCL supports) and the planes are recombined."""
    import torch

    if world <= 1:
        return t
    planes = torch.stack([(t >> b) & 1 for b in range(bits)])
    _all_reduce(planes, group, world, op="max")
    t.copy_(sum(planes[b] << b for b in range(bits)).to(t.dtype))
    return t


class _Done:
    def wait(self):
        return None


def _all_to_all(out, inp, out_splits, in_splits, group, world, async_op=False):
    """all_to_all_single; with async_op the returned handle's wait() orders the caller's stream
    after the exchange (RCCL runs it on its own stream meanwhile).  gloo (host staging) and
    world == 1 complete before returning."""
    import torch.distributed as dist

    if world == 1:
        out.copy_(inp)
        return _Done() if async_op else out
    if _staged(group) and out.device.type != "cpu":
        h = out.cpu()
        dist.all_to_all_single(h, inp.cpu(), out_splits, in_splits, group=group)
        out.copy_(h)
        return _Done() if async_op else out
    if async_op:
        return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=True)
    dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
    return out


def iman_conover_lhs(columns, P, n, group=None, phases=None, flags=None):
    """Correlate K generated LHS columns of an N-row design to the target whose Cholesky
    factor is P (K x K), returning this rank's rows of the result, shape (K, rows).

    columns: list of LHSColumn (same on every rank); flags: optional int32 tensor of K
    non-finite flag words (OR-combined over ranks on return, bits unchanged).  Raises ValueError exactly where
    ImanConover.__call__ does (rank-correlation matrix not positive definite)."""
    import torch

    if group is not None or _dist_initialized():
        import torch.distributed as dist

        world, rank = dist.get_world_size(group), dist.get_rank(group)
    else:
        world, rank = 1, 0
    phases = phases or HipPhases()
    K = len(columns)
    if not (1 <= K <= 128) or n <= K:
        raise ValueError(f"The matrix X must have rows > columns. Got shape: {(n, K)}")
    rb = shard_bounds(n, world)
    row0, nrows = rb[rank], rb[rank + 1] - rb[rank]
    cb = shard_bounds(K, world)
    if flags is None:
        flags = phases.empty(K, "int32").zero_()

    # ---- step 1: scores of the local rows -----------------------------------------------
    # Each rank generates its own strata [row0, row1) of the sorted column, plus stratum
    # row0 - 1 so that adjacent pairs (ties, order) are checked across shard boundaries.
    S = phases.empty((K, nrows))
    first_is_prev = row0 > 0
    seg_t0 = row0 - 1 if first_is_prev else row0
    stats = np.zeros(2 * K, dtype=np.int64)
    segments = []
    for c, col in enumerate(columns):
        seg = phases.sorted_segment(col, n, seg_t0, rb[rank + 1] - seg_t0, flags[c:c + 1])
        stats[2 * c:2 * c + 2] = phases.sorted_check(seg)
        segments.append(seg)
    stats_d = torch.from_numpy(stats).to(S.device)
    stats = _all_reduce(stats_d, group, world).cpu().numpy()
    for c, col in enumerate(columns):
        if stats[2 * c + 1]:
            raise NotImplementedError(f"column {c}: the inverse CDF is not monotone on the LHS grid; the sharded "
                                      "path needs a monotone ppf")
        heads = None
        if stats[2 * c]:  # ties: 'average' ranks from the global run heads
            local = phases.run_heads(segments[c], row0, first_is_prev)
            heads = _all_gather_varlen(local, group, world)
        phases.scores(col, n, row0, nrows, heads, S[c])
    del segments

    # ---- step 2: E from the all-reduced Gram matrix ------------------------------------
    sums = _all_reduce(phases.column_sums(S), group, world)
    means = sums / float(n)
    gram = _all_reduce(phases.centered_gram(S, means), group, world)
    _, L = phases.factor(gram.cpu().numpy(), n)

    # ---- step 3: correlated scores of the local rows ------------------------------------
    phases.apply(S, L, np.asarray(P, dtype=np.float64))

    # ---- step 4: column owners rank their full columns, pipelined -----------------------------
    # Exchange i (i < max k_own) moves the i-th owned column of every owner: its rows from all
    # ranks to the owner (all-to-all), the owner ranks it, and its result rows go back (a second
    # all-to-all).  On RCCL the exchanges run asynchronously on the communicator's stream, so
    # column i + 1's CS arrives and column i - 1's Y leaves while column i is being ranked.
    own = [cb[o + 1] - cb[o] for o in range(world)]
    k_own, m = own[rank], max(own)
    Y = phases.empty((K, nrows))
    rows_of = [rb[s + 1] - rb[s] for s in range(world)]

    def cs_exchange(i):
        owners = [o for o in range(world) if i < own[o]]
        send = torch.cat([S[cb[o] + i] for o in owners]) if owners else phases.empty(0)
        in_splits = [nrows if i < own[o] else 0 for o in range(world)]
        out_splits = [rows_of[s] if i < k_own else 0 for s in range(world)]
        recv = phases.empty(sum(out_splits))
        work = _all_to_all(recv, send, out_splits, in_splits, group, world, async_op=True)
        return recv, work, send

    def y_exchange(i, y_col):
        in_splits = [rows_of[s] if i < k_own else 0 for s in range(world)]
        out_splits = [nrows if i < own[o] else 0 for o in range(world)]
        send = y_col if i < k_own else phases.empty(0)
        recv = phases.empty(sum(out_splits))
        work = _all_to_all(recv, send, out_splits, in_splits, group, world, async_op=True)
        return recv, work, send

    def y_scatter(i, recv):
        off = 0
        for o in range(world):
            if i < own[o]:
                Y[cb[o] + i].copy_(recv[off:off + nrows])
                off += nrows

    pending_cs = cs_exchange(0) if m else None
    pending_y = []
    for i in range(m):
        cur = pending_cs  # (recv, work, send): the send buffer stays referenced until the wait
        pending_cs = cs_exchange(i + 1) if i + 1 < m else None
        recv_cs, work_cs, _ = cur
        work_cs.wait()
        del cur
        y_col = None
        if i < k_own:
            col = columns[cb[rank] + i]
            sorted_full = phases.sorted_segment(col, n, 0, n, flags[cb[rank] + i:cb[rank] + i + 1])
            y_col = phases.empty(n)
            phases.reorder(recv_cs, sorted_full, y_col)
            del sorted_full
        del recv_cs
        pending_y.append((i,) + y_exchange(i, y_col))
        while len(pending_y) > 2:  # bound the buffers in flight
            j, recv_y, work_y, _ = pending_y.pop(0)
            work_y.wait()
            y_scatter(j, recv_y)
    for j, recv_y, work_y, _ in pending_y:
        work_y.wait()
        y_scatter(j, recv_y)
    del S
    _all_reduce_flags(flags, group, world)
    return Y


def _dist_initialized():
    try:
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized()
    except ImportError:
        return False
