"""Per-rank time budget of the row-sharded cfg4 run, emulated on one GPU:
the work one rank r of R does -- steps 1-3 over its N / R rows of all K columns, step 4 of its
K / R owned columns (N rows each), Y of its rows regenerated from the positions -- timed phase
by phase with the exchanges left out (they are priced from the bytes each rank sends).

    python tools/rank_budget.py [--rows 100000000] [--world 8] [--rank 0] [--reps 3]

Prints one JSON line.  The owned columns' correlated scores come from one single-GPU call
(the same CS every rank's all-to-all would deliver)."""

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()

    import ctypes

    import numpy as np
    import torch

    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd import _lib, device
    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.distributed import HEADS_CAP, DISCRETE, HipPhases, LHSColumn, shard_bounds

    n, K = a.rows, 32
    C = cfg3_corr(K)
    P = np.linalg.cholesky(C)
    from probabilit_amd.modeling import _parse_scipy_args

    cols = [LHSColumn(7, c, _lib.DIST_IDS[name], [float(x) for x in _parse_scipy_args(name, (), kw)])
            for c, (name, kw) in enumerate(cfg_dists(K))]
    flags = device.zeros(K, "int32")
    icc = [_lib.ICColumn(7, c, col.dist, (ctypes.c_double * 4)(*col.params), len(col.params),
                         flags.data_ptr() + 4 * c) for c, col in enumerate(cols)]
    CS = device.empty((K, n))
    ImanConover().set_target(C)._transform_generated(icc, n, debug={"CS": CS})
    ph = HipPhases()
    out = {"rows": n, "d": K, "rank": a.rank, "per_world": {}}

    def timed(fn):
        best = 1e30
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
        return round(best * 1e3, 3)

    for world in a.world:
        rb, cb = shard_bounds(n, world), shard_bounds(K, world)
        r = a.rank
        row0, row1 = rb[r], rb[r + 1]
        nrows = row1 - row0
        seg_t0 = row0 - 1 if row0 > 0 else row0
        counts = ph.zeros((K, 2), "int64")
        hcur = ph.zeros(K, "int32")
        heads = ph.empty((K, HEADS_CAP), "int32")
        S = ph.empty((K, nrows))
        owned = list(range(cb[r], cb[r + 1]))
        p_cols = [ph.empty(n, "int32") for _ in owned]
        p_back = torch.randint(0, n, (K, nrows), dtype=torch.int64, device=S.device).to(torch.int32)  # valid positions
        Y = ph.empty((K, nrows))

        def counts_phase():  # discrete: counts + heads; continuous: the (deferred) certificate
            for c, col in enumerate(cols):
                d = col.dist in DISCRETE
                ph.sorted_counts(col, n, seg_t0, row1 - seg_t0, flags[c:c + 1], counts[c],
                                 heads=heads[c] if d else None, hcur=hcur[c:c + 1] if d else None, certify=not d)

        def scores_phase():
            for c, col in enumerate(cols):
                ph.scores(col, n, row0, nrows, None, S[c])

        def gram_phase():
            means = ph.column_sums(S) / float(n)
            ph.centered_gram(S, means)

        L = np.linalg.cholesky(C)  # any factor: the timing does not depend on its values

        def apply_phase():
            ph.apply(S, L, P)

        def owned_phase():
            h = ph.owned_begin([cols[c] for c in owned], n)
            for i, c in enumerate(owned):
                ph.owned_column(h, i, CS[c], p_cols[i], ph.ready(h))
            ph.owned_finish(h)
            ph.owned_end(h)

        def values_phase():
            for c, col in enumerate(cols):
                ph.values_at(col, n, p_back[c], Y[c])

        t = {"counts": timed(counts_phase), "scores": timed(scores_phase), "gram": timed(gram_phase),
             "apply": timed(apply_phase), "owned_step4": timed(owned_phase), "values_at": timed(values_phase)}
        t["compute_total"] = round(sum(t.values()), 3)
        k_own = len(owned)
        # bytes this rank sends (= receives) over xGMI: its rows of the other owners' columns out
        # (8 B), the positions of its owned columns' foreign rows back (4 B)
        out_cs = (K - k_own) * nrows * 8
        out_p = k_own * (n - nrows) * 4
        t["xgmi_bytes_out"] = out_cs + out_p
        out["per_world"][str(world)] = t
        del S, p_cols, p_back, Y, heads
    print(json.dumps(out))


if __name__ == "__main__":
    main()
