"""Benchmark: BASELINE.json metric -- Msamples/s (N x d draws) + achieved HBM GB/s,
LHS + Iman-Conover, d = 32 (config 3: N = 1e8 on one MI355X).

One step = one full `NoOp(*ds).correlate(*ds, corr_mat=C).sample_device(N, method="lhs")`
through the public DAG API: native LHS fused into the 32 inverse-CDF kernels (norm / gamma /
triang / poisson x 4, BASELINE config 2 set), then the Iman-Conover reorder of all 32 columns
(rank + scores + Gram + decorrelate/correlate + rank + gather); outputs stay in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--rows ROWS] [--d COLS] [--cpu-n ROWS]

With N > 1 (torch.distributed.run, one process per GPU, RCCL) the same N-row problem is
row-sharded across the ranks (BASELINE config 4; strong scaling): rank r generates and
scores rows [N r / R, N (r + 1) / R), the Gram matrix is all-reduced, and the step-4 rank
of each column runs on its owner between two all-to-alls (probabilit_amd/distributed.py).
Prints ONE JSON line on rank 0.
"""

import argparse
import json
import re
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 TB/s measured copy)


# Algorithmic HBM bytes per row of ONE launch of each timed kernel (SURVEY.md §8(d) unit
# figures, restated for the kernels this build runs; step 4 = the generated-column path of
# pbh_step4.hip).  A launch covers one column, except the kernels in ALL_COLUMNS (k columns).
LAUNCH_BYTES = {
    "k_lhs_sorted_ppf": 0,       # stratum-ordered generation for the tie / inversion counts only: nothing stored
    "k_perm_scores": 8,          # write S 8 (ranks from the LHS permutation: no sort of X)
    "k_gram": 8,                 # read S 8                                   (all columns)
    "k_apply": 20,               # read S 8, write CS 8 + code 4              (all columns)
    "k_hist16": 4,               # read code 4                                (all columns)
    "k_msd1": 12,                # read code 4, write code 4 + row 4
    "k_msd2": 14,                # read code 4 + row 4, write low16 2 + row 4
    "k_finish": 14,              # bucket finish: read low16 2 + row 4, write (row, p) 8
    "k_place_msd": 16,           # one row-placement MSD pass: read 8 + write 8
    "k_place_gen": 16,           # read (row, p) 8, write Y 8 (sort(X)[p] regenerated, not read)
    # the general path (columns whose codes are not flat, or with runs beyond the finish)
    "k_digit_hist<u32>": 4, "k_scatter<u32>": 16, "k_code_runs": 17, "k_scatter<place>": 24, "k_place": 20,
    "k_lhs_ppf": 8, "k_ppf": 16, "k_elementwise": 24,
}
ALL_COLUMNS = {"k_gram", "k_apply", "k_hist16"}


def kernel_bytes(name, n, k):
    """Algorithmic bytes of ONE launch of `name` over n rows (k columns for ALL_COLUMNS)."""
    return LAUNCH_BYTES.get(name, 0) * n * (k if name in ALL_COLUMNS else 1)


# bench (HIP-event) kernel names -> rocprofv3 kernel names in the committed PMC summaries
PMC_NAMES = {"k_scatter<u32>": ["k_onesweep<unsigned int, unsigned int, 36>", "k_onesweep<unsigned int, unsigned int, 32>",
                                "k_onesweep<unsigned int, unsigned int, 16>", "k_scatter<unsigned int>"],
             "k_scatter<place>": ["k_onesweep<unsigned int, double, 24>", "k_onesweep<unsigned int, double, 16>",
                                  "k_scatter<unsigned int, double>"],
             "k_code_runs": ["k_code_buckets", "k_runs_resolve"], "k_gram": ["k_gram_mfma", "k_gram"],
             "k_apply": ["k_apply_mfma_w2<true>", "k_apply_mfma_w2<false>", "k_apply_mfma", "k_apply<32>"], "k_digit_hist<u32>": ["k_digit_hist<unsigned int>"],
             "k_place": ["k_place"], "k_perm_scores": ["k_perm_scores<false>", "k_perm_scores"],
             "k_finish": ["k_finish_q<2048, 512, false>", "k_finish_q<1024, 512, false>", "k_finish_q<1024, 512, true>", "k_finish_q<2048, 512, true>",
                          "k_finish_q<1024, 256, true>", "k_finish_ah<2048>", "k_finish_ah<1024>", "k_finish_ah<4096>", "k_finish_fused<2, 4096>", "k_finish_fused<2, 4096, false>",
                          "k_finish_fused<2, 4096, true>", "k_finish_fused<1, 4096>", "k_finish_fused<2, 2048>",
                          "k_finish_fused<1, 2048>", "k_finish_fused<4, 2048>", "k_finish_fused<4, 4096>", "k_finish"],
             "k_msd1": ["k_msd1x<1024, 8>", "k_msd1x<256, 16>", "k_msd1o", "k_msd1<true>", "k_msd1<false>", "k_msd1"],
             "k_msd2": ["k_msd2x<1024, 8>", "k_msd2x<512, 8>", "k_msd2w", "k_msd2o", "k_msd2<true>", "k_msd2<false>",
                        "k_msd2"],
             "k_place_msd": ["k_place_msdo", "k_place_msd<true>", "k_place_msd<false>", "k_place_msd"],
             "k_hist16": ["k_hist16", "k_hist16c"],
             # one timing id over every variant that ran (the cfg3 set: norm, lognorm, triang,
             # uniform, expon, gamma, poisson): traffic = their dispatch-weighted mean
             "k_place_gen": ["k_place_gen<0>", "k_place_gen<1>", "k_place_gen<2>", "k_place_gen<3>", "k_place_gen<4>",
                             "k_place_gen_direct<0>", "k_place_gen_direct<3>", "k_place_gen_gamma",
                             "k_place_gen_gamma_w<false>",
                             "k_place_gen_poisson"],
             "k_lhs_sorted_ppf": ["k_lhs_sorted_ppf<0>", "k_lhs_sorted_ppf<1>", "k_lhs_sorted_ppf<2>",
                                  "k_lhs_sorted_ppf<3>", "k_lhs_sorted_ppf<4>", "k_lhs_sorted_ppf<5>",
                                  "k_lhs_sorted_ppf<6>"]}


def _profile_tag(path):
    """Order of committed profiles, newest last (mtimes do not survive a checkout): the round
    directory profiles/r<RR>/, then the pass tag of the file name (`_r77`, `_r3m` < `_r3p`)."""
    d = re.search(r"r(\d+)$", os.path.basename(os.path.dirname(path)))
    m = re.search(r"_r(\d+)([a-z]*)", os.path.basename(path))
    return (int(d.group(1)) if d else -1, int(m.group(1)) if m else -1, m.group(2) if m else "")


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary
    (profiles/r*/pmc_traffic_*.json, written by tools/gpu/pmc.sh + tools/pmc_summary.py:
    2 x FETCH_SIZE + WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md), or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic_*.json")), key=_profile_tag)
    if not files:
        return None, None
    ks = json.load(open(files[-1]))["kernels"]
    names = [nm for nm in PMC_NAMES.get(kernel, [kernel]) if nm in ks]  # the variants that ran
    disp = sum(ks[nm]["dispatches"] for nm in names)
    if not disp:
        return None, None
    per = sum(ks[nm]["hbm_bytes"] * ks[nm]["dispatches"] for nm in names) / disp  # per dispatch (pmc_summary.py)
    return int(per), os.path.relpath(files[-1], ROOT)


def _free_port():
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n):
    """`bench.py --gpus N` started without torch.distributed.run: start N rank processes under it
    as children (before this process touches the GPU: no exec) and exit with their status."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--d", type=int, default=32)
    ap.add_argument("--cpu-n", type=int, default=1_000_000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (D2H included) side measurement")
    ap.add_argument("--ppf-rows", type=int, default=100_000_000, help="rows of the ppf-sweep side measurement (0: skip)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--operator-rows", type=int, default=100_000_000,
                    help="rows of the ImanConover().set_target(C)(X) side measurement (0: skip)")
    ap.add_argument("--refstream-rows", type=int, default=100_000_000,
                    help="rows of the second same-seed (stream='reference') side measurement (0: skip)")
    ap.add_argument("--check-out", default=None,
                    help="write each rank's per-column SHA-1 of its rows of Y (JSON) into this directory")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import numpy as np

    import probabilit_amd  # noqa: F401  (first: it sets the HIP queue count before the runtime starts)
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    backend = None
    if world > 1:
        import torch.distributed as dist

        ndev = torch.cuda.device_count()  # counts devices without initialising the GPU
        local = int(os.environ.get("LOCAL_RANK", "0"))
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
        # one GPU per rank over RCCL; fewer GPUs than ranks (a one-GPU box) rehearses the same
        # sharded path over gloo with the ranks sharing the device (PBH_DIST_BACKEND overrides)
        backend = os.environ.get("PBH_DIST_BACKEND", "nccl" if ndev >= local_world else "gloo")
        torch.cuda.set_device(local % ndev)
        dist.init_process_group(backend)
    else:
        dist = None

    from probabilit_amd import _lib, device
    from probabilit_amd.modeling import Distribution, NoOp

    dev = device.device()
    n, d = args.rows, args.d
    base = [("norm", {"loc": 0.0, "scale": 1.0}), ("gamma", {"a": 2.0}), ("triang", {"c": 0.3}),
            ("poisson", {"mu": 4.0}), ("norm", {"loc": 5.0, "scale": 2.0}), ("gamma", {"a": 0.7, "scale": 3.0}),
            ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}), ("poisson", {"mu": 30.0})]
    dists = (base * ((d + 7) // 8))[:d]
    A = np.random.default_rng(0).normal(size=(64, d))
    C = 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(d)
    ds = [Distribution(name, **kw) for name, kw in dists]
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    group = dist.group.WORLD if dist is not None else None

    def step(i):
        return root.sample_device(n, random_state=args.seed + i, method="lhs", group=group)

    def barrier():
        torch.cuda.synchronize(dev)
        if dist is not None:
            dist.barrier()

    for i in range(args.warmup):
        step(i)
    lib = _lib.load()
    lib.pbh_timing_reset()
    lib.pbh_timing_enable(1)
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
    barrier()
    t1 = time.perf_counter()
    lib.pbh_timing_enable(0)
    elapsed = t1 - t0
    if args.check_out:  # the last timed step's rows of every column (tests compare with one GPU)
        import hashlib

        os.makedirs(args.check_out, exist_ok=True)
        digests = [hashlib.sha1(x.samples_device.cpu().numpy().tobytes()).hexdigest() for x in ds]
        with open(os.path.join(args.check_out, f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "world": world, "rows": n, "seed": args.seed + args.warmup + args.steps - 1,
                       "sha1": digests}, f)
    if dist is not None:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    value = n * d / (ms_per_step / 1e3) / 1e6  # the whole job: N x d draws per step

    # per-kernel device time inside the timed region (HIP events on the launching stream; the
    # step-4 lanes and the deferred counts run concurrently, so these durations are stretched)
    kernels = read_kernels(lib, n, d, args.steps)

    # the standalone pass (outside the timed region): one more step with every kernel on one
    # stream in order (pbh_set_serial: one step-4 lane, counts first), so each launch's duration
    # is its own -- what the committed rocprofv3 1-stream summary measures; the roofline's kernel
    # and duration come from here
    lib.pbh_set_serial(1)
    lib.pbh_timing_reset()
    lib.pbh_timing_enable(1)
    barrier()
    step(args.warmup + args.steps)
    barrier()
    lib.pbh_timing_enable(0)
    lib.pbh_set_serial(0)
    standalone = read_kernels(lib, n, d, 1)
    dom = max(standalone, key=lambda k: standalone[k]["total_ms_per_step"])
    dk = standalone[dom]
    achieved = dk["GBps"] or 0.0
    traffic, traffic_src = pmc_traffic(dom)
    valu, valu_src = pmc_valu(dom)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                "kernel": dom, "avg_launch_ms": dk["avg_ms"], "bytes_per_launch": dk["bytes_per_launch"],
                "duration_source": "standalone pass: pbh_set_serial(1), one stream, HIP events",
                "valu_busy": valu, "valu_source": valu_src}

    # whole-step roofline: SURVEY.md §8(d)'s 96 algorithmic bytes per draw over the step time
    # (the N-row job is row-sharded over `world` GPUs: n * d draws in all, against world x the peak)
    pipeline = {"bytes_per_draw": 96, "achieved": round(96 * n * d / (ms_per_step / 1e3) / 1e9, 1),
                "unit": "GB/s", "peak": HBM_PEAK_GBS * world,
                "frac": round(96 * n * d / (ms_per_step / 1e3) / 1e9 / (HBM_PEAK_GBS * world), 4),
                "kernel_time_ms_per_step": round(sum(k["total_ms_per_step"] for k in standalone.values()), 3),
                "kernel_time_source": "standalone pass (concurrent durations in `kernels` overlap)"}
    copy_peak = hbm_copy_peak(lib) if rank == 0 else None
    if copy_peak:
        pipeline["frac_of_measured_copy"] = round(pipeline["achieved"] / copy_peak["GBps"], 4)
        roofline["frac_of_measured_copy"] = round(achieved / copy_peak["GBps"], 4)
    e2e = end_to_end(root, ds, n, d, args.seed + args.warmup + args.steps, barrier, ms_per_step) \
        if (world == 1 and not args.no_e2e) else None

    same_seed = reference_stream(root, args.seed, barrier) if (world == 1 and not args.no_e2e) else None
    if same_seed is not None and args.refstream_rows > 0:
        same_seed["at_rows"] = reference_stream(root, args.seed + 100, barrier, n=args.refstream_rows, reps=1,
                                                stream_only=False, profile_tag="refstream")
    op = None
    if world == 1 and args.operator_rows > 0:
        for x in ds:  # the cfg3 result is no longer needed: its HBM goes to the operator's X and Y
            del x.samples_
        op = operator_ic(ds, C, args.operator_rows, args.seed + 200, barrier, lib)

    sweep = ppf_sweep(lib, base, args.ppf_rows, args.seed) if (args.ppf_rows > 0 and rank == 0) else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_n, d)

    if rank == 0:
        line = {"metric": "Msamples/s (N\u00d7d draws) + achieved HBM GB/s, LHS+ImanConover d=32",  # BASELINE.json
                "value": round(value, 2),
                "unit": "Msamples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
                "scaling": "strong" if world > 1 else "weak",
                "vs_baseline": None, "dtype": "f64", "data": "synthetic (native LHS quantiles, seeded)",
                "config": {"workload": ("cfg4: " if world > 1 else "cfg3: ") +
                                       "d=32 (cfg2 set x4), LHS + ppf + ImanConover, N rows",
                           "rows": n, "d": d,
                           "parallelism": (f"row-sharded x{world} ({backend}: all-reduce + all-to-all of scores "
                                           "out, positions back)") if world > 1 else "single",
                           "devices": torch.cuda.device_count() if world > 1 else 1},
                "roofline": roofline, "pipeline_roofline": pipeline, "hbm_copy_peak": copy_peak,
                "end_to_end": e2e, "reference_stream": same_seed, "operator_ic": op, "cpu_baseline": cpu, "ppf_sweep": sweep, "kernels": kernels,
                "kernels_standalone": standalone}
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def read_kernels(lib, n, d, steps):
    """Per-kernel HIP-event totals since the last pbh_timing_reset, per step."""
    import ctypes

    from probabilit_amd import _lib

    kernels = {}
    for kid, name in enumerate(_lib.KERNELS):
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(tot), ctypes.byref(cnt)))
        if cnt.value:
            avg = tot.value / cnt.value
            b = kernel_bytes(name, n, d)
            kernels[name] = {"total_ms_per_step": round(tot.value / steps, 3), "launches": cnt.value,
                             "avg_ms": round(avg, 4), "bytes_per_launch": b,
                             "GBps": round(b / (avg / 1e3) / 1e9, 1) if b else None}
    return kernels


def pmc_valu(kernel):
    """VALU-busy of `kernel` (the share of SIMD cycles that issued a vector instruction,
    tools/pmc_valu_summary.py) from the newest committed rocprofv3 VALU pass, dispatch-weighted
    over the kernel's template variants, or None."""
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_valu_*.json")), key=_profile_tag)
    for f in reversed(files):
        ks = json.load(open(f)).get("runs", {}).get("bench", {})
        names = [nm for nm in PMC_NAMES.get(kernel, [kernel]) if nm in ks]
        disp = sum(ks[nm]["dispatches"] for nm in names)
        if disp:
            v = sum(ks[nm]["valu_busy"] * ks[nm]["dispatches"] for nm in names) / disp
            return round(v, 3), os.path.relpath(f, ROOT)
    return None, None


# the sweep kernel each cfg2 distribution takes (pbh_ppf.hip launch_ppf), for its VALU-busy figure
SWEEP_KERNELS = {"norm": "k_ppf_c<0, true>", "lognorm": "k_ppf_c<3, true>", "gamma": "k_ppf_gamma_w<false>",
                 "poisson": "k_ppf_poisson_lds", "triang": "k_ppf_v<4>", "uniform": "k_ppf_v<1>",
                 "expon": "k_ppf_v<2>"}


def ppf_sweep(lib, dists, n, seed, reps=3):
    """Side measurement for the north_star's "ppf sweep" roofline (16 B/draw, read
    q 8 + write x 8, at the sample_from_quantiles boundary): pbh_ppf over one HBM-resident
    quantile column of n rows for each cfg2 distribution, HIP-event time of k_ppf on the
    launching stream.  Not part of `value` (the fused LHS path never stores q)."""
    import ctypes

    from probabilit_amd import _lib, native

    q = native.fill_uniform(seed + 12345, n, 1, return_device=True)[0]
    kid = _lib.KERNELS.index("k_ppf")
    per, tot_ms, tot_b = {}, 0.0, 0
    # ~70 ms of untimed launches first: the sweep follows seconds of host work (CPU baseline, end to
    # end) with the GPU idle, and the first distribution otherwise ran ~10% slow at lowered clocks
    name0, kw0 = dists[0]
    for _ in range(100):
        native.ppf(name0, q, return_device=True, **kw0)
    for name, kw in dists:
        for _ in range(2):  # warm: the tables built once, clocks up (the first distribution ran ~7% slow with one)
            native.ppf(name, q, return_device=True, **kw)
        lib.pbh_timing_reset()
        lib.pbh_timing_enable(1)
        for _ in range(reps):
            native.ppf(name, q, return_device=True, **kw)
        lib.pbh_timing_enable(0)
        t, c = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(t), ctypes.byref(c)))
        avg = t.value / max(c.value, 1)
        ent = {"ms": round(avg, 4), "GBps": round(16 * n / (avg / 1e3) / 1e9, 1)}
        kname = SWEEP_KERNELS.get(name)
        if kname:  # issue-level bound next to the bandwidth (committed rocprofv3 VALU pass)
            valu, src = pmc_valu(kname)
            if valu is not None:
                bound = ("HBM" if ent["GBps"] >= 0.6 * HBM_PEAK_GBS else "VALU" if valu >= 0.7
                         else "latency (VALU-busy < 0.7, < 0.6 of HBM)")
                ent.update({"kernel": kname, "valu_busy": valu, "valu_source": src, "bound": bound})
        per[f"{name}{kw}"] = ent
        tot_ms += avg
        tot_b += 16 * n
    gbps = tot_b / (tot_ms / 1e3) / 1e9
    return {"kernel": "k_ppf", "rows": n, "bytes_per_draw": 16, "achieved": round(gbps, 1), "unit": "GB/s",
            "frac": round(gbps / HBM_PEAK_GBS, 4), "per_dist": per}


def hbm_copy_peak(lib, nbytes=4 << 30, reps=5):
    """The box's HBM copy ceiling (re-measure with a copy kernel and report it
    next to the 8 TB/s spec): the fastest of pbh_hbm_copy's variants over nbytes, read + write
    bytes / mean launch time."""
    import ctypes

    import torch

    from probabilit_amd import _lib, device

    src = torch.empty(nbytes, dtype=torch.uint8, device=device.device())
    dst = torch.empty_like(src)
    src.fill_(1)
    kid = _lib.KERNELS.index("k_hbm_copy")
    per = {}
    for var in range(5):
        _lib.check(lib.pbh_hbm_copy(src.data_ptr(), dst.data_ptr(), nbytes, var, device.stream()))
        lib.pbh_timing_reset()
        lib.pbh_timing_enable(1)
        for _ in range(reps):
            _lib.check(lib.pbh_hbm_copy(src.data_ptr(), dst.data_ptr(), nbytes, var, device.stream()))
        lib.pbh_timing_enable(0)
        t, c = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(t), ctypes.byref(c)))
        per[var] = t.value / max(c.value, 1)
    del src, dst
    best = min(per, key=per.get)
    avg = per[best]
    return {"kernel": "k_hbm_copy", "bytes_moved": 2 * nbytes, "variant": best, "avg_ms": round(avg, 4),
            "GBps": round(2 * nbytes / (avg / 1e3) / 1e9, 1),
            "frac_of_spec": round(2 * nbytes / (avg / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "per_variant_GBps": {v: round(2 * nbytes / (ms / 1e3) / 1e9, 1) for v, ms in per.items()}}


def end_to_end(root, ds, n, d, seed, barrier, device_ms):
    """The drop-in call end to end: Node.sample() (the reference's API, modeling.py:431) leaves a
    numpy samples_ on every node (modeling.py:582-583, 614), here all 32 columns handed back in one
    pipelined batch through the pinned ring (device.to_host_many).  d2h = the total minus the
    device-resident step time measured above.  A side figure, never `value`."""
    from probabilit_amd import device

    barrier()
    t0 = time.perf_counter()
    root.sample(n, random_state=seed, method="lhs")
    host = [x.samples_ for x in ds]
    t1 = time.perf_counter()
    nbytes = sum(h.nbytes for h in host)
    del host
    ms = (t1 - t0) * 1e3
    d2h_ms = max(ms - device_ms, 1e-3)
    return {"value": round(n * d / (ms / 1e3) / 1e6, 2), "unit": "Msamples/s", "ms": round(ms, 1),
            "device_ms": round(device_ms, 1), "d2h_ms": round(d2h_ms, 1),
            "d2h_GBps": round(nbytes / (d2h_ms / 1e3) / 1e9, 2), "bytes": nbytes,
            "what": f"Node.sample() with numpy samples_ on all columns (pinned-ring D2H, "
                    f"{device.__dict__['_STAGE_BYTES'] >> 20} MiB chunks)"}


def reference_stream(root, seed, barrier, n=10_000_000, reps=2, stream_only=True, profile_tag=None):
    """The same-seed mode (stream="reference": scipy's LatinHypercube(d, rng=seed) stream bit for
    bit, modeling.py:480,488 -> scipy _random_lhs) on the cfg3 graph at N = 1e7, device-resident
    output: the device PCG64 uniforms, the d Fisher-Yates shuffles decoded on the device
    (pbh_lhs_reference -> pbh_lhs_dev.hip: banded classification, a host walk of the ambiguous
    draws, an exact check of every decision, permutations from the swap targets), then the same
    ppf + Iman-Conover through the general (materialised) path.  A side figure."""
    import ctypes

    from probabilit_amd import _lib

    root.sample_device(n, random_state=seed, method="lhs", stream="reference")  # warm (workspaces)
    barrier()
    t0 = time.perf_counter()
    for i in range(reps):
        root.sample_device(n, random_state=seed + 1 + i, method="lhs", stream="reference")
    barrier()
    ms = (time.perf_counter() - t0) / reps * 1e3
    d = root.num_distribution_nodes()
    dev, att, amb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int64()
    _lib.check(_lib.load().pbh_lhs_reference_stats(ctypes.byref(dev), ctypes.byref(att), ctypes.byref(amb)))
    if not stream_only:
        out = {"value": round(n * d / (ms / 1e3) / 1e6, 2), "unit": "Msamples/s", "ms": round(ms, 1), "rows": n, "d": d,
               "reps": reps, "shuffles_on_device": bool(dev.value), "decode_attempts": att.value,
               "ambiguous_draws": amb.value}
        if profile_tag:
            out["dominant_kernel"] = committed_profile(profile_tag, n)
        return out
    # the stream alone: scipy's LatinHypercube(d, rng=seed).random(n) matrix, device-resident
    from probabilit_amd import qmc

    barrier()
    t0 = time.perf_counter()
    for i in range(reps):
        qmc.make_source("lhs", n, d, seed + 11 + i, stream="reference").matrix()
    barrier()
    ms_stream = (time.perf_counter() - t0) / reps * 1e3
    return {"value": round(n * d / (ms / 1e3) / 1e6, 2), "unit": "Msamples/s", "ms": round(ms, 1), "rows": n, "d": d,
            "stream_only": {"value": round(n * d / (ms_stream / 1e3) / 1e6, 2), "unit": "Msamples/s",
                            "ms": round(ms_stream, 1),
                            "what": "LatinHypercube(d, rng=seed).random(n) alone (uniforms + shuffles + combine)"},
            "shuffles_on_device": bool(dev.value), "decode_attempts": att.value, "ambiguous_draws": amb.value,
            "what": "Node.sample_device(1e7, method='lhs', stream='reference'): same results as the reference on "
                    "the same seed (the shuffle stream decoded on the device), then ppf + Iman-Conover"}


# Algorithmic bytes per row of one launch of the materialised-X path's kernels (the reference
# operator ImanConover()(X) on an (N, K) C-order X; pbh_iman_conover with X given): the step-1
# sort of each column (k_load_keys, k_digit_hist, the 64-bit one-sweep passes k_scatter, the
# rank finish), then the general step 4 (32-bit code passes, runs, row placement).
OPERATOR_BYTES = {
    "k_load_keys": 16,            # read X 8 (stride K), write key 8
    "k_digit_hist": 8,            # read key 8
    "k_scatter": 20,              # one 64-bit pass: read key 8 (+ row 4 after the first), write key 8 + row 4 -- 20 counted
    "k_rank_finish<scores>": 24,  # read key 8 + row 4, write S 8 (+ sorted X 8 would be 32; 24 counted)
    "k_gram": 8, "k_apply": 20, "k_digit_hist<u32>": 4, "k_scatter<u32>": 16, "k_code_runs": 17,
    "k_scatter<place>": 24, "k_place": 20, "k_rank_finish<gather>": 24,
}
OPERATOR_ALL_COLUMNS = {"k_gram", "k_apply"}


def committed_profile(tag, n):
    """The dominant kernel (largest total duration) of the newest committed one-stream rocprofv3
    kernel-stats summary profiles/r*/rocprof_<tag>_*.csv (tools/side_profile.py <tag>), with its
    mean duration; None when none is committed."""
    import csv
    import glob

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", f"rocprof_{tag}_*.csv")), key=_profile_tag)
    if not files:
        return None
    rows = list(csv.DictReader(open(files[-1])))
    top = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    return {"kernel": top["Name"], "calls": int(top["Calls"]), "avg_ms": round(float(top["AverageNs"]) / 1e6, 4),
            "share_of_kernel_time": round(float(top["TotalDurationNs"]) / total, 4),
            "source": os.path.relpath(files[-1], ROOT)}


def operator_ic(ds, C, n, seed, barrier, lib, reps=2):
    """The reference operator itself, ImanConover().set_target(C)(X) (correlation.py:368-425),
    on a device-resident materialised (n, K) C-order X: the cfg3 leaves sampled uncorrelated (the
    X the reference's sample_from_quantiles stacks, modeling.py:577-578), then the general path
    -- a 64-bit radix sort of every column for step 1, the scores, Gram, step 3, the code sort and
    row placement of step 4 -- returning a new (n, K) Y.  A side figure, not `value`; per-kernel
    standalone durations (one stream, HIP events) give the dominant kernel's roofline."""
    import torch

    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.modeling import NoOp

    K = len(ds)
    NoOp(*ds).sample_device(n, random_state=seed, method="lhs")
    X = torch.stack([x.samples_device for x in ds], dim=1)  # (n, K) C-order, as np.vstack(...).T
    for x in ds:
        del x.samples_
    inst = ImanConover().set_target(C)
    Y = inst(X)  # warm (workspace, code map)
    del Y
    barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        Y = inst(X)
        del Y
    barrier()
    ms = (time.perf_counter() - t0) / reps * 1e3
    # one more call with every kernel on one stream in order, each launch timed on its own
    lib.pbh_set_serial(1)
    lib.pbh_timing_reset()
    lib.pbh_timing_enable(1)
    Y = inst(X)
    barrier()
    lib.pbh_timing_enable(0)
    lib.pbh_set_serial(0)
    del Y, X
    import ctypes

    from probabilit_amd import _lib

    per = {}
    for kid, name in enumerate(_lib.KERNELS):
        tot, cnt = ctypes.c_double(), ctypes.c_int64()
        _lib.check(lib.pbh_timing_read(kid, ctypes.byref(tot), ctypes.byref(cnt)))
        if cnt.value:
            avg = tot.value / cnt.value
            b = OPERATOR_BYTES.get(name, 0) * n * (K if name in OPERATOR_ALL_COLUMNS else 1)
            per[name] = {"total_ms": round(tot.value, 3), "launches": cnt.value, "avg_ms": round(avg, 4),
                         "bytes_per_launch": b, "GBps": round(b / (avg / 1e3) / 1e9, 1) if b else None}
    dom = max(per, key=lambda k: per[k]["total_ms"]) if per else None
    roof = None
    if dom and per[dom]["GBps"]:
        roof = {"kernel": dom, "avg_launch_ms": per[dom]["avg_ms"], "bytes_per_launch": per[dom]["bytes_per_launch"],
                "achieved": per[dom]["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(per[dom]["GBps"] / HBM_PEAK_GBS, 4)}
    return {"value": round(n * K / (ms / 1e3) / 1e6, 2), "unit": "Msamples/s", "ms": round(ms, 1), "rows": n, "d": K,
            "reps": reps, "roofline": roof, "kernels_standalone": per,
            "kernel_time_ms": round(sum(v["total_ms"] for v in per.values()), 3),
            "rocprof": committed_profile("operator", n),
            "what": "ImanConover().set_target(C)(X) on a device-resident (N, K) C-order X (the reference's "
                    "operator API, correlation.py:368-425): new Y, X unchanged"}


def cpu_baseline(n, d):
    """The reference's CPU path (oracle.pipeline: scipy LatinHypercube -> scipy ppf ->
    Iman-Conover restated in numpy with the reference's calls) on this host, at N = n rows
    (default 1e6: the size BASELINE.md quotes, 0.90 Msamples/s on the survey's 8-core Xeon)."""
    import math

    from threadpoolctl import threadpool_info

    from oracle.pipeline import lhs_ic

    t0 = time.perf_counter()
    lhs_ic(n, d, 0)
    dt = time.perf_counter() - t0
    threads = max([p.get("num_threads", 1) for p in threadpool_info()] or [1])
    rate = n * d / dt / 1e6
    # the work per draw grows like log N (two sorts per column), so the rate at 1e8 is labelled
    # an N log N extrapolation from the measured N, not a measurement
    extrap = rate * math.log(n) / math.log(1e8)
    return {"value": round(rate, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "openblas_num_threads": os.environ.get("OPENBLAS_NUM_THREADS"),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "survey_value_at_1e6": 0.90,
            "extrapolated_1e8": {"value": round(extrap, 4), "method": f"N log N from N={n}: rate x ln({n}) / ln(1e8)"},
            "sample": f"cfg3 at N={n}, d={d} ({dt:.1f} s): scipy LHS + scipy ppf + numpy/scipy Iman-Conover; "
                      f"ppf/sort single-threaded, BLAS pool of {threads} threads (cores = that pool)"}


if __name__ == "__main__":
    main()
