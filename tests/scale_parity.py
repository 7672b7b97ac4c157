"""Helpers for the at-scale parity gates of the headline path; used by
tests/test_gpu_scale.py and tools/parity_1e8.py.  The device side runs the production
Iman-Conover path of Node.sample(method="lhs") on natively generated cfg3 columns; the
reference side recomputes the correlated scores the reference's way (correlation.py:398-414:
np.corrcoef, np.linalg.cholesky, scipy.linalg.solve_triangular, then @ P.T), ranks them
(rankdata(...).astype(int) - 1, correlation.py:422) and counts the step-4 index mismatches.
Two legs: scores="device" starts from the device's step-1 scores S; scores="reference" runs the
reference's step 1 as well (correlation.py:394-395): X = scipy.stats ppf of the same native
quantiles (modeling.py:807), rankdata(X, 'average') / (N + 1), scipy.special.ndtri."""

import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def cfg3_generated(n, d, seed, C):
    """The cfg3 graph's correlated columns exactly as Node._evaluate hands them to
    ImanConover._transform_generated (modeling.py fast path): returns (inst, columns, flags)."""
    from probabilit_amd import _lib, device, qmc
    from probabilit_amd.correlation import ImanConover, nearest_correlation_matrix
    from probabilit_amd.modeling import Distribution

    import ctypes

    from oracle.pipeline import cfg_dists

    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    inst = ImanConover().set_target(nearest_correlation_matrix(C))
    flags = device.zeros(d, "int32")
    s = qmc.seed_from(seed)
    cols = []
    for j, v in enumerate(ds):
        params = [float(p) for p in v._params(n)]
        cols.append(_lib.ICColumn(s, j, _lib.DIST_IDS[v.distr], (ctypes.c_double * 4)(*params), len(params),
                                  flags.data_ptr() + 4 * j))
    return inst, cols, flags


def run_device(n, d, seed, C):
    """Production path with the step-1 scores S, the step-3 correlated scores CS and E kept:
    returns (Y, S, CS) device (K, N) blocks, E (host K x K), P and the column descriptors."""
    from probabilit_amd import device

    inst, cols, _ = cfg3_generated(n, d, seed, C)
    dbg = {"S": device.empty((d, n)), "CS": device.empty((d, n)), "E": np.zeros((d, d))}
    Y = inst._transform_generated(cols, n, debug=dbg)
    device.synchronize()
    return Y, dbg["S"], dbg["CS"], dbg["E"], np.asarray(inst.P), cols


def sorted_x(col, n):
    """np.sort(X[:, k]) of a generated column (correlation.py:423): the stratum-ordered
    generator's output (pbh_lhs_sorted_ppf), host array.  The device output column is not a
    permutation of it where the device saw an exact CS tie, so it cannot be rebuilt by sorting Y."""
    from probabilit_amd import _lib, device

    out, flag = device.empty(n), device.zeros(1, "int32")
    _lib.check(_lib.load().pbh_lhs_sorted_ppf(col.seed, n, 0, n, col.lhs_col, col.dist, col.params, col.nparams,
                                              out.data_ptr(), flag.data_ptr(), device.stream()), "pbh_lhs_sorted_ppf")
    return device.to_host(out)


def reference_cs(S, E, P, k=None):
    """CS the reference's way from scores S (host (K, N), i.e. the reference's S.T) and E:
    L = cholesky(E); D = solve_triangular(L, S.T, lower=True).T; CS = D @ P.T
    (correlation.py:405-414).  With k, only the first k columns (the lower-triangular solve
    and P make them depend on the first k score columns only).  Returns (N, k)."""
    import scipy.linalg

    L = np.linalg.cholesky(E)
    K = S.shape[0] if k is None else k
    D = scipy.linalg.solve_triangular(L[:K, :K], S[:K], lower=True).T
    return D @ np.asarray(P)[:K, :K].T


def _rank_minus_one(cs):
    """rankdata(cs).astype(int) - 1 (correlation.py:422) via the oracle restatement."""
    from oracle.ic import rankdata_average

    return rankdata_average(cs).astype(np.int64) - 1


def column_gate(k, cs_ref, y_dev, sx, cs_dev=None, tol=1e-13):
    """Step-4 mismatches of one column.  y_dev is the device's output column, a permutation of
    the sorted column sx (or, where the device saw an exact CS tie, a column with that tie's
    repeated value, as rankdata's 'average' + astype(int) gives); the reference output is
    sx[rank(cs_ref) - 1].  Every row where they differ must sit at an adjacent reference rank:
    its device value is sx at reference rank +-1, and the row holding that rank has a
    reference CS within `tol` of this row's.  Such a pair is a "swap" when the partner got this
    row's reference value, or a "tie" when the device gave both rows the same value (the
    device's CS tied exactly where the reference's differ by an ulp, or the reverse).
    Returns a dict (counts, worst |dCS|, violations)."""
    t0 = time.time()
    r = _rank_minus_one(cs_ref)
    n = r.shape[0]
    y_ref = sx[r]
    bad = np.flatnonzero(y_ref != y_dev)
    out = {"column": int(k), "rows": int(n), "mismatched_rows": int(bad.size), "swaps": 0, "ties": 0,
           "max_abs_dcs_ref": 0.0, "violations": 0, "seconds": None}
    if bad.size:
        counts = np.bincount(r, minlength=n)
        inv = None
        if counts.max() == 1:  # no reference tie: one row per rank
            inv = np.empty(n, dtype=np.int64)
            inv[r] = np.arange(n, dtype=np.int64)

        def rows_at(p):
            return [int(inv[p])] if inv is not None else [int(i) for i in np.flatnonzero(r == p)]

        viol, swaps, ties, worst = 0, set(), set(), 0.0
        detail = []
        for row in bad:
            v = y_dev[row]
            kind = None
            for step in (-1, 0, 1):  # step 0: a reference tie (several rows share one rank)
                p = r[row] + step
                if not (0 <= p < n) or sx[p] != v:
                    continue
                for partner in rows_at(p):
                    if partner == row:
                        continue
                    dcs = abs(float(cs_ref[row]) - float(cs_ref[partner]))
                    if dcs >= tol:
                        continue
                    pair = (min(row, partner), max(row, partner))
                    if y_dev[partner] == sx[r[row]]:
                        kind = "swap"
                        swaps.add(pair)
                    elif y_dev[partner] == v:
                        kind = "tie"
                        ties.add(pair)
                    else:
                        continue
                    worst = max(worst, dcs)
                    if len(detail) < 8:
                        d = {"row": int(row), "partner": int(partner), "kind": kind, "abs_dcs_ref": dcs}
                        if cs_dev is not None:
                            d["abs_dcs_dev"] = abs(float(cs_dev[row]) - float(cs_dev[partner]))
                        detail.append(d)
                    break
                if kind:
                    break
            g = int(counts[r[row]])
            if not kind and g > 1:
                # a reference tie group (equal CS): rankdata's 'average' gives all g rows the index
                # p = int(avg) - 1 of sorted positions [a, a + g); where the device's CS differ by an
                # ulp it hands the group those g distinct values instead
                p = int(r[row])
                a = p + 1 - (g + 1) // 2
                if sx[a] <= v <= sx[a + g - 1]:
                    partners = [int(i) for i in np.flatnonzero(r == p) if i != row]
                    dcs = max(abs(float(cs_ref[row]) - float(cs_ref[q])) for q in partners)
                    if dcs < tol:
                        kind = "ref_tie"
                        ties.add(tuple(sorted([int(row)] + partners)))
                        worst = max(worst, dcs)
                        if len(detail) < 8:
                            detail.append({"row": int(row), "partners": partners, "kind": kind, "abs_dcs_ref": dcs,
                                           "group": g})
            viol += 0 if kind else 1
        out.update(swaps=len(swaps), ties=len(ties), max_abs_dcs_ref=worst, violations=viol, pairs=detail)
        if cs_dev is not None:
            out["max_abs_cs_dev_minus_ref_on_mismatches"] = float(np.max(np.abs(cs_dev[bad] - cs_ref[bad])))
    out["seconds"] = round(time.time() - t0, 1)
    return out


def gate(cs_ref_cols, y_cols, sx_cols, cs_dev_cols=None, threads=4, log=None):
    """column_gate over columns; cs_ref_cols (N, k), y_cols / sx_cols / cs_dev_cols: lists of host (N,)."""
    k = cs_ref_cols.shape[1]

    def one(j):
        res = column_gate(j, np.ascontiguousarray(cs_ref_cols[:, j]), y_cols[j], sx_cols[j],
                          None if cs_dev_cols is None else cs_dev_cols[j])
        if log:
            log(res)
        return res

    with ThreadPoolExecutor(max(1, min(threads, k))) as ex:
        return list(ex.map(one, range(k)))


def _chunked(fn, x, threads, chunk=1 << 22):
    """fn over row chunks of a 1-D array on a thread pool (numpy / scipy ufuncs release the GIL)."""
    out = np.empty(x.shape[0])

    def run(r0):
        out[r0:r0 + chunk] = fn(x[r0:r0 + chunk])

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(run, range(0, x.shape[0], chunk)))
    return out


def reference_scores(col, name, kw, n, threads=16):
    """The reference's step 1 for one generated column (correlation.py:394-395) from the reference's
    own values: X = scipy.stats.<name>(**kw).ppf(q) of the column's native quantiles q
    (modeling.py:807), ranks = rankdata(X, 'average'), S = ndtri(ranks / (N + 1)).

    The ranks are taken in stratum order: the device sorts the quantiles (torch.sort, which also
    gives the row of every stratum), scipy's ppf runs on them in that order, and where its values
    never decrease, rankdata(X) is the stratum position, averaged over each run of equal values --
    the same numbers rankdata's argsort gives, without a 10^8-element sort per column.  A decrease
    (a non-monotone scipy ppf) falls back to scipy.stats.rankdata on the row-order X.
    Returns (S in row order, host (N,), info dict)."""
    import scipy.special
    import scipy.stats
    import torch

    from oracle.ppf import ppf
    from probabilit_amd import _lib, device

    q = device.empty(n)
    _lib.check(_lib.load().pbh_fill_lhs(col.seed, n, 0, n, col.lhs_col, 1, q.data_ptr(), n, device.stream()))
    qs, order = torch.sort(q)
    del q
    qs_h, order_h = device.to_host(qs), order.cpu().numpy()
    del qs, order
    xs = _chunked(lambda v: ppf(name, v, **kw), qs_h, threads)
    del qs_h
    dx = np.diff(xs)
    info = {"column": int(col.lhs_col), "dist": name, "params": kw, "ties": int(np.count_nonzero(dx == 0)),
            "decreases": int(np.count_nonzero(dx < 0))}
    if info["decreases"]:
        xrow = np.empty(n)
        xrow[order_h] = xs
        rank_row = scipy.stats.rankdata(xrow)
    else:
        if info["ties"]:
            starts = np.concatenate([[0], np.flatnonzero(dx != 0) + 1])
            ends = np.concatenate([starts[1:], [n]])
            rank_t = np.repeat((starts + 1 + ends) / 2.0, ends - starts)  # 'average' over each run
        else:
            rank_t = np.arange(1, n + 1, dtype=np.float64)
        rank_row = np.empty(n)
        rank_row[order_h] = rank_t
    del xs, dx, order_h
    return _chunked(lambda v: scipy.special.ndtri(v / (n + 1)), rank_row, threads), info


def gate_all(n, d, seed, C, threads=8, log=print, scores="device"):
    """The §8(d) gate over every column (tools/parity_1e8.py, tests/test_gpu_scale.py): the
    production path on the device keeping S, then on the host E = np.corrcoef(S)
    (correlation.py:398), L = cholesky(E), D = solve_triangular(L, S.T).T, CS = D @ P.T
    (:405-414), the reference ranks (:422) and, per column, every row whose device output
    differs from sort(X[:, k])[idx].  Returns the summary document."""
    from probabilit_amd import device

    t0 = time.time()
    Y, S, CS, E_dev, P, gen = run_device(n, d, seed, C)
    extra = {}
    if scores == "reference":
        from oracle.pipeline import cfg_dists

        S_dev = S
        S_ref = np.empty((n, d))  # the reference's S: (N, K), C order (correlation.py:395)
        infos, worst_s = [], 0.0
        for j, (name, kw) in enumerate(cfg_dists(d)):
            sj, info = reference_scores(gen[j], name, kw, n, threads=threads)
            info["max_abs_s_dev_minus_ref"] = float(np.max(np.abs(device.to_host(S_dev[j]) - sj)))
            worst_s = max(worst_s, info["max_abs_s_dev_minus_ref"])
            S_ref[:, j] = sj
            del sj
            infos.append(info)
            log(f"[{time.time() - t0:6.1f}s] reference step 1, column {j}: {info}")
        del S_dev, S
        E_ref = np.corrcoef(S_ref, rowvar=False)  # correlation.py:398, on the reference's own scores
        log(f"[{time.time() - t0:6.1f}s] max |E_dev - E_ref| = {float(np.max(np.abs(E_dev - E_ref))):.3e}")
        import scipy.linalg

        L = np.linalg.cholesky(E_ref)  # correlation.py:405-414, literally
        cs_ref = scipy.linalg.solve_triangular(L, S_ref.T, lower=True).T @ np.asarray(P).T
        del S_ref
        extra = {"step1": infos, "max_abs_s_dev_minus_ref": worst_s}
    else:
        S_host = device.to_host(S)
        del S
        E_ref = np.corrcoef(S_host.T, rowvar=False)  # the reference's S is (N, K): S_host.T
        log(f"[{time.time() - t0:6.1f}s] max |E_dev - E_ref| = {float(np.max(np.abs(E_dev - E_ref))):.3e}")
        cs_ref = reference_cs(S_host, E_ref, P)
        del S_host
    log(f"[{time.time() - t0:6.1f}s] reference CS done")

    def one(j):
        y = device.to_host(Y[j])
        csd = device.to_host(CS[j])
        r = column_gate(j, np.ascontiguousarray(cs_ref[:, j]), y, sorted_x(gen[j], n), csd)
        r["max_abs_cs_dev_minus_ref"] = float(np.max(np.abs(csd - cs_ref[:, j])))
        log(r)
        return r

    import threading

    done = []
    stop = threading.Event()

    def heartbeat():  # a line a minute: long gates are not mistaken for hung runs
        while not stop.wait(60):
            log(f"[{time.time() - t0:6.1f}s] {len(done)} of {d} columns gated")

    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        with ThreadPoolExecutor(threads) as ex:
            cols = []
            for r in ex.map(one, range(d)):
                cols.append(r)
                done.append(r["column"])
    finally:
        stop.set()
    what = ("SURVEY.md §8(d) step-4 parity gate: device (production path) vs the reference's "
            + ("own steps 1-4: scipy ppf of the native quantiles, rankdata/(N+1), ndtri, corrcoef, cholesky, "
               "solve_triangular, @P.T, rankdata" if scores == "reference" else
               "corrcoef/cholesky/solve_triangular/@P.T/rankdata on the device scores S"))
    return {"what": what, "scores": scores, **extra,
            "workload": f"cfg3 (cfg2 set x4), N={n}, d={d}, native LHS seed {seed}, "
                        "target C = 0.9 corrcoef(A) + 0.1 I",
            "rows": n, "d": d, "seed": seed,
            "max_abs_E_dev_minus_ref": float(np.max(np.abs(E_dev - E_ref))),
            "mismatched_rows_total": sum(c["mismatched_rows"] for c in cols),
            "swaps_total": sum(c["swaps"] for c in cols),
            "ties_total": sum(c["ties"] for c in cols),
            "violations_total": sum(c["violations"] for c in cols),
            "max_abs_dcs_ref_in_swaps": max(c["max_abs_dcs_ref"] for c in cols),
            "max_abs_cs_dev_minus_ref": max(c["max_abs_cs_dev_minus_ref"] for c in cols),
            "seconds": round(time.time() - t0, 1), "columns": cols}
