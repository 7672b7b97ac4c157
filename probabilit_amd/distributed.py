"""Row-sharded multi-GPU Iman-Conover over natively generated LHS columns.

One process per GPU (torch.distributed, backend "nccl" = RCCL on ROCm).  Rank r of R owns
the rows [N r / R, N (r + 1) / R) of every column and the columns [K o / R, K (o + 1) / R)
for step 4.  The reference's single-process ImanConover.__call__ (correlation.py:368-425)
is split where its data dependencies cross rows:

    step 1  the tie / inversion counts of each column's strata in this shard (counted, not
            stored; the pair across a shard boundary counted once), summed over ranks by one
            all-reduce; a discrete column's run heads from every shard, one all-gather of the
            (short) sorted lists; then the scores of the local rows from the LHS permutation
            (no sort).
    step 2  column sums, then the centered Gram matrix of the local rows; each summed over
            ranks by an all-reduce (K and K x K doubles), then E = corrcoef and
            L = cholesky(E) on every rank's host (identical inputs -> identical L).
    step 3  CS = S L^-T P^T on the local rows.
    step 4  per owned-column index i, one all-to-all brings the i-th owned column of every
            owner from the row shards (8 bytes a row); the owner ranks it with the single-GPU
            step-4 passes (pbh_ic_owned_*: codes, top-16 histogram with the adaptive code map,
            MSD code passes, bucket finish, row placement) into the sorted position p of every
            row; a second all-to-all sends the positions back (4 bytes a row); every rank then
            regenerates its rows of Y = sort(X)[p] (pbh_lhs_values_at) -- sort(X) of a generated
            column is a function of p, so no value crosses a link.

On RCCL every all-to-all is asynchronous on the communicator's stream and ordered with the
library's step-4 lanes by events: column i + 1's scores arrive while column i is ranked, and
column i's positions leave as soon as its lane finishes.

The returned block is this rank's rows of every correlated column, (K, rows) on its GPU.
The compute of every phase goes through a `phases` object: `HipPhases` (the C-ABI of
libprobabilit_hip) in production; tests substitute a CPU implementation to exercise the
exchange logic under the gloo backend on machines without a GPU.
"""

import ctypes

import numpy as np

from . import _lib, device

HEADS_CAP = 16384  # run heads a discrete column's shard may append (kHeadsCap, pbh_step4.h)
DISCRETE = {_lib.DIST_IDS[d] for d in ("poisson", "binom", "bernoulli", "geom", "randint", "nbinom", "dlaplace",
                                        "planck", "boltzmann")}  # sorted columns with runs


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

    def ic_column(self):
        return _lib.ICColumn(self.seed, self.lhs_col, self.dist, (ctypes.c_double * 4)(*self.params),
                             len(self.params), None)


class _Owned:
    """A pbh_ic_owned handle with its workspace and the events it handed out."""

    def __init__(self, handle, ws, cols):
        self.handle = handle
        self.ws = ws
        self.cols = cols
        self.events = []


class HipPhases:
    """The Iman-Conover phases of include/probabilit_hip.h on this process's GPU."""

    def __init__(self):
        self.lib = _lib.load()
        self.dev = device.device()

    # -- allocation helpers -------------------------------------------------------------
    def empty(self, shape, dtype="float64"):
        return device.empty(shape, dtype)

    def zeros(self, shape, dtype="float64"):
        return device.zeros(shape, dtype)

    def _ws(self, nbytes):
        return device.empty(max(int(nbytes), 256), "uint8")

    # -- stream ordering ------------------------------------------------------------------
    def _event(self):
        ev = ctypes.c_void_p()
        _lib.check(self.lib.pbh_event_create(ctypes.byref(ev)), "pbh_event_create")
        return ev

    def ready(self, owned):
        """An event recorded on the current stream (its work so far), owned by `owned`."""
        ev = self._event()
        owned.events.append(ev)
        _lib.check(self.lib.pbh_event_record(ev, device.stream()), "pbh_event_record")
        return ev

    def wait(self, ev, stream=None):
        """`stream` (default: the current one) continues after event `ev`."""
        if ev is not None:
            _lib.check(self.lib.pbh_stream_wait_event(stream if stream is not None else device.stream(), ev),
                       "pbh_stream_wait_event")

    # -- step 1 ---------------------------------------------------------------------------
    def sorted_counts(self, col, n, t0, nt, flag, counts, heads=None, hcur=None, certify=False):
        prm = (ctypes.c_double * 4)(*col.params)
        _lib.check(self.lib.pbh_lhs_sorted_counts(col.seed, n, t0, nt, col.lhs_col, col.dist, prm, len(col.params),
                                                  counts.data_ptr(), heads.data_ptr() if heads is not None else None,
                                                  hcur.data_ptr() if hcur is not None else None,
                                                  heads.shape[0] if heads is not None else 0, flag.data_ptr(),
                                                  int(certify), device.stream()), "pbh_lhs_sorted_counts")

    def sort_heads(self, heads):
        _lib.check(self.lib.pbh_sort_heads(heads.data_ptr(), heads.shape[0], device.stream()), "pbh_sort_heads")

    def segment_heads(self, col, n, t0, nt, first_is_prev, flag):
        """Run heads of strata [t0, t0 + nt) from the materialised segment (the rare fallback:
        a continuous column that ties, or a discrete one with more heads than HEADS_CAP)."""
        out = device.empty(max(nt, 1))
        prm = (ctypes.c_double * 4)(*col.params)
        _lib.check(self.lib.pbh_lhs_sorted_ppf(col.seed, n, t0, nt, col.lhs_col, col.dist, prm, len(col.params),
                                               out.data_ptr(), flag.data_ptr(), device.stream()),
                   "pbh_lhs_sorted_ppf")
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_run_heads_workspace_size(nt, ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        heads = device.empty(max(nt, 1), "int32")
        count = ctypes.c_int64()
        _lib.check(self.lib.pbh_run_heads(out.data_ptr(), nt, t0 + 1 if first_is_prev else t0, int(first_is_prev),
                                          heads.data_ptr(), ctypes.byref(count), ws.data_ptr(), nbytes.value,
                                          device.stream()), "pbh_run_heads")
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
    def owned_begin(self, cols, n):
        arr = (_lib.ICColumn * len(cols))(*[c.ic_column() for c in cols])
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_ic_owned_workspace_size(n, len(cols), ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        h = ctypes.c_void_p()
        _lib.check(self.lib.pbh_ic_owned_create(arr, len(cols), n, ws.data_ptr(), nbytes.value, ctypes.byref(h),
                                                device.stream()), "pbh_ic_owned_create")
        return _Owned(h, ws, arr)

    def owned_column(self, owned, i, cs, p_out, ready):
        """Rank column i of `owned` from its full correlated scores cs into the positions
        p_out (after event `ready`); returns the event recorded when p_out is complete."""
        done = self._event()
        owned.events.append(done)
        _lib.check(self.lib.pbh_ic_owned_column(owned.handle, i, cs.data_ptr(), None, 1, p_out.data_ptr(), ready, done,
                                                device.stream()), "pbh_ic_owned_column")
        return done

    def owned_finish(self, owned):
        """Join the lanes; the indices of the columns the general path redid (their positions
        changed after their done events)."""
        m = len(owned.cols)
        redone = np.zeros(m, dtype=np.int32)
        _lib.check(self.lib.pbh_ic_owned_finish(owned.handle, redone.ctypes.data, device.stream()),
                   "pbh_ic_owned_finish")
        return [i for i in range(m) if redone[i]]

    def owned_end(self, owned):
        _lib.check(self.lib.pbh_ic_owned_destroy(owned.handle, device.stream()), "pbh_ic_owned_destroy")
        for ev in owned.events:
            self.lib.pbh_event_destroy(ev)
        owned.events = []

    def values_at(self, col, n, p, y):
        """y[r] = sort(X[:, col])[p[r]] for the rows of this shard."""
        c = col.ic_column()
        _lib.check(self.lib.pbh_lhs_values_at(ctypes.byref(c), n, p.data_ptr(), p.shape[0], y.data_ptr(), 1,
                                              device.stream()), "pbh_lhs_values_at")

    # -- materialised columns on their owner (iman_conover_block) --------------------------
    def column_scores(self, x, s_out, sx_out, flag):
        """Step 1 of a whole materialised column: s_out = ndtri(rankdata(x) / (n + 1)),
        sx_out = np.sort(x); a NaN sets flag."""
        n = x.shape[0]
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_rank_workspace_size(n, ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        _lib.check(self.lib.pbh_ic_column_scores(x.data_ptr(), 1, n, s_out.data_ptr(), sx_out.data_ptr(),
                                                 flag.data_ptr(), ws.data_ptr(), nbytes.value, device.stream()),
                   "pbh_ic_column_scores")

    def reorder(self, cs, sx, y):
        """Step 4 of a whole column: y = sx[rankdata(cs).astype(int) - 1]."""
        n = cs.shape[0]
        nbytes = ctypes.c_size_t()
        _lib.check(self.lib.pbh_ic_reorder_workspace_size(n, ctypes.byref(nbytes)))
        ws = self._ws(nbytes.value)
        _lib.check(self.lib.pbh_ic_reorder(cs.data_ptr(), n, sx.data_ptr(), y.data_ptr(), 1, None, ws.data_ptr(),
                                           nbytes.value, device.stream()), "pbh_ic_reorder")


def _solo(world):
    """world == 1 skips the collectives -- unless PBH_FORCE_COLLECTIVES=1, which runs them on a
    one-rank communicator (tests: the RCCL calls, streams and events on a one-GPU box)."""
    import os

    return world == 1 and os.environ.get("PBH_FORCE_COLLECTIVES") != "1"


def _staged(group):
    """gloo moves host memory only: device tensors are staged through the host for it
    (used when several ranks share one GPU, e.g. in tests); RCCL/NCCL moves them in place."""
    import torch.distributed as dist

    return dist.get_backend(group) == "gloo"


def _all_gather_varlen(t, group, world, sizes=None):
    """Concatenation over ranks (in rank order) of 1-D tensors of different lengths (`sizes`,
    when every rank already knows them, saves one exchange)."""
    import torch
    import torch.distributed as dist

    if _solo(world):
        return t
    dev = t.device
    if _staged(group):
        t = t.cpu()
    if sizes is None:
        size = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        got = [torch.zeros_like(size) for _ in range(world)]
        dist.all_gather(got, size, group=group)
        sizes = [int(s.item()) for s in got]
    m = max(max(sizes), 1)
    padded = torch.zeros(m, dtype=t.dtype, device=t.device)
    padded[:t.shape[0]] = t
    parts = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)]).to(dev)


def _all_gather_rows(t, group, world):
    """(world, *t.shape) stack of every rank's `t` (same shape everywhere)."""
    import torch
    import torch.distributed as dist

    if _solo(world):
        return t[None]
    dev = t.device
    src = t.cpu() if _staged(group) else t
    parts = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(parts, src, group=group)
    return torch.stack(parts).to(dev)


def _all_reduce(t, group, world, op="sum"):
    import torch.distributed as dist

    if not _solo(world):
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


def _exchange(out_list, in_list, group, world, phases, after=None, side_stream=None):
    """All-to-all of tensor lists (in_list[d] goes to rank d, out_list[s] comes from rank s).
    `after`: an event the exchange must wait for (a lane's done event).  On RCCL the exchange is
    asynchronous on the communicator's stream -- issued from `side_stream` when `after` is given,
    so that the caller's stream is not held back -- and the returned handle's wait() orders the
    caller's stream after it.  gloo (host staging) and world == 1 complete before returning."""
    import torch
    import torch.distributed as dist

    if _solo(world):
        phases.wait(after)
        out_list[0].copy_(in_list[0])
        return _Done()
    if _staged(group):
        phases.wait(after)  # the host copy below synchronises the current stream, now after `after`
        hin = torch.cat([t.reshape(-1) for t in in_list]).cpu()
        hout = torch.empty(sum(t.numel() for t in out_list), dtype=hin.dtype)
        dist.all_to_all_single(hout, hin, [t.numel() for t in out_list], [t.numel() for t in in_list], group=group)
        off = 0
        for t in out_list:
            t.copy_(hout[off:off + t.numel()].view(t.shape))
            off += t.numel()
        return _Done()
    if after is None:
        return dist.all_to_all(out_list, in_list, group=group, async_op=True)
    with torch.cuda.stream(side_stream):
        phases.wait(after, side_stream.cuda_stream)
        return dist.all_to_all(out_list, in_list, group=group, async_op=True)


class _Redo(Exception):
    """A deferred tie / inversion count was non-zero: the scores assumed untied are wrong."""


def iman_conover_lhs(columns, P, n, group=None, phases=None, flags=None, defer=None):
    """Correlate K generated LHS columns of an N-row design to the target whose Cholesky
    factor is P (K x K), returning this rank's rows of the result, shape (K, rows).

    columns: list of LHSColumn (same on every rank); flags: optional int32 tensor of K
    non-finite flag words (OR-combined over ranks on return, bits unchanged).  Raises ValueError exactly where
    ImanConover.__call__ does (rank-correlation matrix not positive definite).

    defer (default: on for the HIP phases, PBH_DEFER_COUNTS=0 turns it off): the continuous
    columns' tie / inversion counts -- an event of probability ~1e-8 per column at N = 1e8 --
    run on a side stream after step 3, next to the first exchange and the owners' ranking,
    their scores computed as untied; the summed counts are checked at the end and a non-zero
    one (on any rank: the sum is global) redoes the call with every count first, as the
    single-GPU call does (pbh_iman_conover, PBH_DEFER_COUNTS)."""
    import os

    if group is not None or _dist_initialized():
        import torch.distributed as dist

        world, rank = dist.get_world_size(group), dist.get_rank(group)
    else:
        world, rank = 1, 0
    phases = phases or HipPhases()
    if defer is None:
        defer = isinstance(phases, HipPhases) and os.environ.get("PBH_DEFER_COUNTS", "3") != "0"
    K = len(columns)
    if n <= K:
        raise ValueError(f"The matrix X must have rows > columns. Got shape: {(n, K)}")
    if not 1 <= K <= 128:
        raise ValueError(f"Iman-Conover on the device takes 1 to 128 variables, got {K}")
    if flags is None:
        flags = phases.zeros(K, "int32")
    # every attempt flags into a scratch word per column; the caller's words are OR-ed with the
    # attempt that stands, so bits set before the call are kept and a redone attempt's are not doubled
    if defer:
        scratch = phases.zeros(K, "int32")
        try:
            Y = _iman_conover_lhs(columns, P, n, group, world, rank, phases, scratch, True)
            flags |= scratch
            return Y
        except _Redo:
            pass
    scratch = phases.zeros(K, "int32")
    Y = _iman_conover_lhs(columns, P, n, group, world, rank, phases, scratch, False)
    flags |= scratch
    return Y


def _iman_conover_lhs(columns, P, n, group, world, rank, phases, flags, defer):
    import torch

    K = len(columns)
    rb = shard_bounds(n, world)
    row0, row1 = rb[rank], rb[rank + 1]
    nrows = row1 - row0
    cb = shard_bounds(K, world)

    # ---- step 1: tie / inversion counts of every column's strata in this shard ----------
    # The segment starts one stratum early (row0 - 1) so that the pair across the shard
    # boundary is counted here, and only here; a discrete column also appends its run heads.
    first_is_prev = row0 > 0
    seg_t0 = row0 - 1 if first_is_prev else row0
    seg_len = row1 - seg_t0
    disc = [c for c, col in enumerate(columns) if col.dist in DISCRETE]
    late = [c for c in range(K) if defer and c not in disc]  # counted after step 3
    counts = phases.zeros((K, 2), "int64")
    hcur = phases.zeros(K, "int32")
    heads_buf = phases.empty((max(len(disc), 1), HEADS_CAP), "int32")
    for c, col in enumerate(columns):
        if c in late:
            continue
        hb = heads_buf[disc.index(c)] if c in disc else None
        phases.sorted_counts(col, n, seg_t0, seg_len, flags[c:c + 1], counts[c], heads=hb,
                             hcur=hcur[c:c + 1] if hb is not None else None)
    stats = _all_reduce(counts, group, world).cpu().numpy()
    hc_all = _all_gather_rows(hcur, group, world).cpu().numpy()  # (world, K) appended heads per shard

    S = phases.empty((K, nrows))
    for c, col in enumerate(columns):
        if stats[c, 1]:
            raise NotImplementedError(f"column {c}: the inverse CDF is not monotone on the LHS grid; the sharded "
                                      "path needs a monotone ppf")
        heads = None
        if stats[c, 0]:  # ties: 'average' ranks from the global run heads
            if c in disc and hc_all[:, c].max() <= HEADS_CAP:
                local = heads_buf[disc.index(c)][:int(hc_all[rank, c])]
                phases.sort_heads(local)
                heads = _all_gather_varlen(local, group, world, sizes=[int(v) for v in hc_all[:, c]])
            else:
                local = phases.segment_heads(col, n, seg_t0, seg_len, first_is_prev, flags[c:c + 1])
                heads = _all_gather_varlen(local, group, world)
        phases.scores(col, n, row0, nrows, heads, S[c])
    del heads_buf

    # ---- step 2: E from the all-reduced Gram matrix ------------------------------------
    sums = _all_reduce(phases.column_sums(S), group, world)
    means = sums / float(n)
    gram = _all_reduce(phases.centered_gram(S, means), group, world)
    _, L = phases.factor(gram.cpu().numpy(), n)

    # ---- step 3: correlated scores of the local rows ------------------------------------
    phases.apply(S, L, np.asarray(P, dtype=np.float64))

    # the deferred counts, on a side stream next to the exchanges and the owners' ranking
    cstream = None
    if late:
        dcounts = phases.zeros((K, 2), "int64")
        if isinstance(phases, HipPhases):
            cstream = torch.cuda.Stream(device=S.device)
            cstream.wait_stream(torch.cuda.current_stream(S.device))
        with torch.cuda.stream(cstream) if cstream is not None else _nullcontext():
            for c in late:  # the certificate: only a non-zero sum (possible tie) redoes with exact counts
                phases.sorted_counts(columns[c], n, seg_t0, seg_len, flags[c:c + 1], dcounts[c], certify=True)

    # ---- step 4: column owners rank their full columns, pipelined -----------------------------
    own = [cb[o + 1] - cb[o] for o in range(world)]
    k_own, m = own[rank], max(own)
    cs_cols = [phases.empty(n) for _ in range(k_own)]  # owned columns' scores, all rows
    p_cols = [phases.empty(n, "int32") for _ in range(k_own)]  # their sorted positions, all rows
    p_back = phases.empty((K, nrows), "int32")  # this shard's positions in every column
    Y = phases.empty((K, nrows))
    owned = phases.owned_begin(columns[cb[rank]:cb[rank + 1]], n) if k_own else None
    nothing = phases.empty(0)
    nothing32 = phases.empty(0, "int32")

    def cs_lists(i):
        send = [S[cb[o] + i] if i < own[o] else nothing for o in range(world)]
        recv = [cs_cols[i][rb[s]:rb[s + 1]] if i < k_own else nothing for s in range(world)]
        return recv, send

    def p_lists(i):
        send = [p_cols[i][rb[s]:rb[s + 1]] if i < k_own else nothing32 for s in range(world)]
        recv = [p_back[cb[o] + i] if i < own[o] else nothing32 for o in range(world)]
        return recv, send

    def values(i):  # Y of this shard in every owner's i-th column: sort(X)[p] regenerated
        for o in range(world):
            if i < own[o]:
                c = cb[o] + i
                phases.values_at(columns[c], n, p_back[c], Y[c])

    side = None
    if not _solo(world) and not _staged(group):
        side = torch.cuda.Stream(device=S.device)
        side.wait_stream(torch.cuda.current_stream(S.device))
    try:
        # every scores exchange up front (the communicator runs them in order); then per column:
        # rank it when its scores are in, send its positions back when its lane is done, and
        # regenerate this shard's Y of every owner's i-th column when those positions are in
        cs_work = [_exchange(*cs_lists(i), group, world, phases) for i in range(m)]
        p_work = []
        for i in range(m):
            cs_work[i].wait()
            done = None
            if i < k_own:
                done = phases.owned_column(owned, i, cs_cols[i], p_cols[i], phases.ready(owned))
            p_work.append(_exchange(*p_lists(i), group, world, phases, after=done, side_stream=side))
        for i in range(m):
            p_work[i].wait()
            values(i)
        redone = phases.owned_finish(owned) if owned is not None else []
        # a column the fast passes rejected was redone after its positions left: send it again
        again = phases.zeros(max(m, 1), "int32")
        for i in redone:
            again[i] = 1
        again = _all_reduce(again, group, world, op="max").cpu().numpy()
        for i in range(m):
            if again[i]:
                _exchange(*p_lists(i), group, world, phases).wait()
                values(i)
    finally:
        if owned is not None:
            phases.owned_end(owned)
    del cs_cols, p_cols, S

    if late:  # the deferred counts, summed over every rank's segments
        if cstream is not None:
            torch.cuda.current_stream(Y.device).wait_stream(cstream)
        dstats = _all_reduce(dcounts, group, world).cpu().numpy()
        if dstats.any():
            raise _Redo()
    _all_reduce_flags(flags, group, world)
    return Y


def _world(group):
    if group is not None or _dist_initialized():
        import torch.distributed as dist

        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _column_exchanges(n, K, world, rank, phases):
    """The two all-to-all directions of a column-owner exchange over K row-sharded columns:
    to_owner(i, src, dst): every rank's rows of each owner's i-th column (src[c]: this shard's
    rows of column c) land in the owner's whole-column buffer dst[i]; from_owner(i, src, dst) is
    the way back (src[i]: the owner's whole column, dst[c]: this shard's rows of column c)."""
    rb, cb = shard_bounds(n, world), shard_bounds(K, world)
    own = [cb[o + 1] - cb[o] for o in range(world)]
    k_own = own[rank]

    def to_owner(i, src, dst, nothing):
        send = [src[cb[o] + i] if i < own[o] else nothing for o in range(world)]
        recv = [dst[i][rb[s]:rb[s + 1]] if i < k_own else nothing for s in range(world)]
        return recv, send

    def from_owner(i, src, dst, nothing):
        send = [src[i][rb[s]:rb[s + 1]] if i < k_own else nothing for s in range(world)]
        recv = [dst[cb[o] + i] if i < own[o] else nothing for o in range(world)]
        return recv, send

    return to_owner, from_owner, k_own, max(own)


def iman_conover_block(block, P, n, group=None, phases=None):
    """Iman-Conover (correlation.py:368-425) of a row-sharded MATERIALISED block: block is this
    rank's rows (K, rows) of X (shards by shard_bounds), the result this rank's rows of Y.  The
    correlators' other sources -- Sobol', Halton, MT19937 / PCG64 quantiles, the reference LHS
    stream, composite parameters -- take this path (natively generated LHS columns take
    iman_conover_lhs).  Rank r owns columns [K r / R, K (r + 1) / R):

        step 1  X's owned columns to their owner (all-to-all, 8 B a row); the owner ranks each
                whole column ('average' ties) into its scores and keeps np.sort(X[:, k])
                (pbh_ic_column_scores); the scores back to the row shards (8 B a row)
        step 2  column sums and the centered Gram matrix all-reduced; E, L on every host
        step 3  CS = S L^-T P^T on the local rows
        step 4  CS's owned columns to their owner (8 B); the owner reorders its sorted X by the
                ranks of CS (pbh_ic_reorder); Y's rows back to the row shards (8 B)

    No rank holds more than its owned columns whole (K / R x N), and no correlator work is
    replicated.  Raises ValueError exactly where ImanConover.__call__ does (NaN input, rank
    correlation not positive definite)."""
    world, rank = _world(group)
    phases = phases or HipPhases()
    K, nrows = block.shape
    if n <= K:
        raise ValueError(f"The matrix X must have rows > columns. Got shape: {(n, K)}")
    if not 1 <= K <= 128:
        raise ValueError(f"Iman-Conover on the device takes 1 to 128 variables, got {K}")
    to_owner, from_owner, k_own, m = _column_exchanges(n, K, world, rank, phases)
    nothing = phases.empty(0)

    # ---- step 1 on the owners -------------------------------------------------------------
    whole = [phases.empty(n) for _ in range(k_own)]
    for i in range(m):
        _exchange(*to_owner(i, block, whole, nothing), group, world, phases).wait()
    sx = [phases.empty(n) for _ in range(k_own)]
    flag = phases.zeros(1, "int32")
    for i in range(k_own):  # the scores overwrite X's column in place (it is sorted into sx first)
        phases.column_scores(whole[i], whole[i], sx[i], flag)
    if int(_all_reduce(flag, group, world, op="max").cpu()[0]):
        from .correlation import _NOT_PD_MSG

        raise ValueError(_NOT_PD_MSG)  # NaN ranks: corrcoef -> NaN -> not PD (correlation.py:399-403)
    S = phases.empty((K, nrows))
    for i in range(m):
        _exchange(*from_owner(i, whole, S, nothing), group, world, phases).wait()

    # ---- steps 2 and 3 on the row shards ----------------------------------------------------
    sums = _all_reduce(phases.column_sums(S), group, world)
    gram = _all_reduce(phases.centered_gram(S, sums / float(n)), group, world)
    try:
        _, L = phases.factor(gram.cpu().numpy(), n)
    except ValueError:
        from .correlation import _NOT_PD_MSG

        raise ValueError(_NOT_PD_MSG) from None
    phases.apply(S, L, np.asarray(P, dtype=np.float64))

    # ---- step 4 on the owners ---------------------------------------------------------------
    for i in range(m):
        _exchange(*to_owner(i, S, whole, nothing), group, world, phases).wait()
    del S
    ys = [phases.empty(n) for _ in range(k_own)]
    for i in range(k_own):
        phases.reorder(whole[i], sx[i], ys[i])
    del whole, sx
    Y = phases.empty((K, nrows))
    for i in range(m):
        _exchange(*from_owner(i, ys, Y, nothing), group, world, phases).wait()
    return Y


def block_stats(block, n, group=None, phases=None):
    """Column means and the centered Gram matrix sum_r (x_r - mean)(x_r - mean)^T of a
    row-sharded block over all n rows (the np.mean / np.cov inputs of the Cholesky correlator,
    correlation.py:255-285, and of decorrelate): two all-reduces, no rows exchanged."""
    world, _ = _world(group)
    phases = phases or HipPhases()
    sums = _all_reduce(phases.column_sums(block), group, world)
    mean = sums / float(n)
    gram = _all_reduce(phases.centered_gram(block, mean), group, world)
    return mean.cpu().numpy(), gram.cpu().numpy()


def gather_to_root(block, n, group, root=0):
    """The whole (K, n) block on rank `root` (None elsewhere): one all-to-all in which every
    rank sends its rows to the root only.  For correlators whose result depends on state a rank
    cannot share by construction (an unseeded PermutationCorrelator's rng, a user class): they
    run once, on the root, and scatter_from_root hands every rank its rows."""
    world, rank = _world(group)
    phases = HipPhases() if block.is_cuda else _HostPhases()
    rb = shard_bounds(n, world)
    K = block.shape[0]
    full = phases.empty((K, n)) if rank == root else None
    nothing = phases.empty(0)
    for j in range(K):
        send = [block[j] if d == root else nothing for d in range(world)]
        recv = [full[j][rb[s]:rb[s + 1]] if rank == root else nothing for s in range(world)]
        _exchange(recv, send, group, world, phases).wait()
    return full


def scatter_from_root(full, K, n, group, like, root=0):
    """Every rank's rows (K, rows) of the root's (K, n) block `full` (the inverse of gather_to_root)."""
    world, rank = _world(group)
    phases = HipPhases() if like.is_cuda else _HostPhases()
    rb = shard_bounds(n, world)
    out = phases.empty((K, rb[rank + 1] - rb[rank]))
    nothing = phases.empty(0)
    for j in range(K):
        send = [full[j][rb[d]:rb[d + 1]] if rank == root else nothing for d in range(world)]
        recv = [out[j] if s == root else nothing for s in range(world)]
        _exchange(recv, send, group, world, phases).wait()
    return out


class _HostPhases:
    """Allocation and (no-op) stream ordering for CPU tensors (gloo tests of the root exchanges)."""

    def empty(self, shape, dtype="float64"):
        import torch

        return torch.empty(shape, dtype=getattr(torch, dtype))

    def wait(self, ev, stream=None):
        pass


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


def _dist_initialized():
    try:
        import torch.distributed as dist

        return dist.is_available() and dist.is_initialized()
    except ImportError:
        return False
