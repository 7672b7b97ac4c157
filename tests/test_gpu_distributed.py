"""The row-sharded Iman-Conover (probabilit_amd/distributed.py) with the HIP phases:

* world size 1: bit-identical to the single-call pbh_iman_conover fast path;
* world size 2 on one GPU (two processes, gloo staging through the host): every rank's rows
  equal the same rows of the single-call result — this exercises the row-offset phases
  (scores of rows [row0, row1), the shard-boundary stratum of the run heads, column owners).
"""

import ctypes
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SPECS = {
    # the cfg2 set: continuous columns and poisson columns with runs (run heads from every shard)
    "cfg2": [(0, [0.0, 1.0]), (5, [2.0, 0.0, 1.0]), (4, [0.3, 0.0, 1.0]), (6, [4.0, 0.0]), (0, [5.0, 2.0]),
             (5, [0.7, 0.0, 3.0]), (4, [0.8, 1.0, 2.0]), (6, [30.0, 0.0])],
    # a leading poisson column: its correlated score IS its tied scores (runs of equal codes beyond
    # the finish), so the owner's fast passes reject it and the general path redoes it
    "tied_first": [(6, [4.0, 0.0]), (0, [0.0, 1.0]), (5, [2.0, 0.0, 1.0]), (4, [0.3, 0.0, 1.0])],
    # extended distributions (pbh_ppf_ext.hip generated columns): PERT's beta, binom / bernoulli
    # run heads by binary search in every shard, truncnorm and a closed form
    "ext": [(7, [3.4, 2.6, 0.0, 10.0]), (9, [20.0, 0.3, 0.0]), (0, [0.0, 1.0]), (10, [0.25, 0.0]),
            (8, [-1.0, 2.0, 1.0, 1.0]), (11, [1.7, 0.0, 1.0])],
}
SPEC = SPECS["cfg2"]
N = 300_007
SEED = 12345


def _target(k=len(SPEC)):
    from oracle.pipeline import cfg3_corr

    return cfg3_corr(k)


def _single_call(spec=SPEC):
    from probabilit_amd import _lib, device
    from probabilit_amd.correlation import ImanConover

    flags = device.zeros(len(spec), "int32")
    cols = [_lib.ICColumn(SEED, c, d, (ctypes.c_double * 4)(*p), len(p), flags.data_ptr() + 4 * c)
            for c, (d, p) in enumerate(spec)]
    Y = ImanConover().set_target(_target(len(spec)))._transform_generated(cols, N)
    return device.to_host(Y)


def _columns(spec=SPEC):
    from probabilit_amd.distributed import LHSColumn

    return [LHSColumn(SEED, c, d, p) for c, (d, p) in enumerate(spec)]


@pytest.mark.parametrize("spec", sorted(SPECS))
def test_world1_matches_single_call(gpu, spec):
    """The sharded orchestration on one rank (owned-column step 4 with positions sent back and
    Y regenerated from them) equals the single-call fast path bit for bit."""
    from probabilit_amd import device
    from probabilit_amd.distributed import iman_conover_lhs

    sp = SPECS[spec]
    ref = _single_call(sp)
    Y = iman_conover_lhs(_columns(sp), np.linalg.cholesky(_target(len(sp))), N)
    np.testing.assert_array_equal(device.to_host(Y), ref)


def test_owned_columns_values_and_positions(gpu):
    """pbh_ic_owned_* directly: a column ranked into Y (gen_place) and the same column ranked
    into positions p then regenerated (pbh_lhs_values_at) agree, and equal the single call;
    the tied leading column is reported redone by the general path."""
    import torch

    from probabilit_amd import _lib, device
    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.distributed import HipPhases

    sp = SPECS["tied_first"]
    cols = _columns(sp)
    lib = _lib.load()
    flags = device.zeros(len(sp), "int32")
    icc = [_lib.ICColumn(SEED, c, d, (ctypes.c_double * 4)(*p), len(p), flags.data_ptr() + 4 * c)
           for c, (d, p) in enumerate(sp)]
    inst = ImanConover().set_target(_target(len(sp)))
    CS = device.empty((len(sp), N))
    Yref = device.to_host(inst._transform_generated(icc, N, debug={"CS": CS}))
    ph = HipPhases()
    for mode in ("y", "p"):
        owned = ph.owned_begin(cols, N)
        Y = device.empty((len(sp), N))
        P = device.empty((len(sp), N), "int32")
        for i in range(len(sp)):
            done = ph._event()
            owned.events.append(done)
            yp = Y[i].data_ptr() if mode == "y" else None
            pp = P[i].data_ptr() if mode == "p" else None
            _lib.check(lib.pbh_ic_owned_column(owned.handle, i, CS[i].data_ptr(), yp, 1, pp, None, done,
                                               device.stream()))
        redone = ph.owned_finish(owned)
        ph.owned_end(owned)
        assert redone == [0]
        if mode == "p":
            for c, col in enumerate(cols):
                ph.values_at(col, N, P[c], Y[c])
        torch.cuda.synchronize()
        np.testing.assert_array_equal(device.to_host(Y), Yref)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, spec="cfg2", backend="gloo"):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    if backend == "nccl":
        torch.cuda.set_device(0)
    dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        from probabilit_amd import device
        from probabilit_amd.distributed import iman_conover_lhs

        sp = SPECS[spec]
        Y = iman_conover_lhs(_columns(sp), np.linalg.cholesky(_target(len(sp))), N, group=dist.group.WORLD)
        np.save(os.path.join(outdir, f"y{rank}.npy"), device.to_host(Y))
    finally:
        dist.destroy_process_group()


class SeededPermutation:
    """correlator=PermutationCorrelator with a fixed seed (the DAG calls correlator() without
    arguments): the one-process result is reproducible, so every rank's rows can be compared."""

    def __new__(cls):
        from probabilit_amd.correlation import PermutationCorrelator

        return PermutationCorrelator(seed=11, iterations=40)


class UnseededPermutation:
    def __new__(cls):
        from probabilit_amd.correlation import PermutationCorrelator

        return PermutationCorrelator(iterations=40)  # seed=None: a fresh rng per instance


class ReverseRows:
    """A user correlator class (the reference's (N, K) ndarray protocol): reverses the rows."""

    def set_target(self, C):
        self.C = C
        return self

    def __call__(self, X):
        return X[::-1].copy()


def _dag(kind):
    from oracle.pipeline import cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    if kind == "correlated":
        ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
        return NoOp(*ds).correlate(*ds, corr_mat=_target()), "lhs"
    if kind == "ext":  # PERT, binom, bernoulli, a closed form: generated columns too
        from probabilit_amd import distributions as dists

        ds = [dists.PERT(0, 6, 10), Distribution("binom", n=20, p=0.3), Distribution("bernoulli", p=0.25),
              Distribution("weibull_min", c=1.7), dists.PERT(1, 2, 9, gamma=10),
              Distribution("binom", n=12, p=0.6, loc=0.5)]  # non-integer loc: the exact count path
        return NoOp(*ds).correlate(*ds, corr_mat=_target(len(ds))), "lhs"
    if kind in ("sobol_ic", "cholesky", "ref_ic", "permcorr", "permcorr_unseeded", "user"):  # materialised block
        ds = [Distribution("norm", loc=1.0, scale=2.0), Distribution("gamma", a=2.0), Distribution("beta", a=2.0, b=3.0),
              Distribution("poisson", mu=4.0)]
        C = np.array([[1.0, 0.5, 0.3, 0.2], [0.5, 1.0, 0.4, 0.1], [0.3, 0.4, 1.0, 0.3], [0.2, 0.1, 0.3, 1.0]])
        return NoOp(*ds).correlate(*ds, corr_mat=C), "sobol" if kind == "sobol_ic" else "lhs"
    if kind == "refstream":  # the reference's own LHS stream: each rank decodes it whole, keeps its rows
        ds = [Distribution("norm", loc=1.0, scale=2.0), Distribution("gamma", a=2.0), Distribution("beta", a=2.0, b=3.0)]
        return NoOp(*ds), "lhs"
    r = 0
    for _ in range(20):  # README mutual-fund loop (BASELINE config 5)
        r = r * Distribution("norm", loc=1.11, scale=0.15) + 1200
    return r, "sobol"


_DAG_KINDS = ("correlated", "fund", "ext", "refstream", "sobol_ic", "cholesky", "ref_ic", "permcorr", "user",
              "permcorr_unseeded")
_DAG_KW = {"refstream": {"stream": "reference"}, "ref_ic": {"stream": "reference"}, "cholesky": {"correlator": "cholesky"},
           "permcorr": {"correlator": SeededPermutation}, "permcorr_unseeded": {"correlator": UnseededPermutation},
           "user": {"correlator": ReverseRows}}


def _dag_worker(rank, world, port, outdir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from probabilit_amd import device

        for kind in _DAG_KINDS:
            root, method = _dag(kind)
            out = root.sample_device(1 << 16, random_state=7, method=method, group=dist.group.WORLD,
                                     **_DAG_KW.get(kind, {}))
            if kind == "fund":
                np.save(os.path.join(outdir, f"{kind}{rank}.npy"), device.to_host(out))
            else:
                for j, d in enumerate(root.get_parents()):
                    np.save(os.path.join(outdir, f"{kind}{rank}_v{j}.npy"), d.samples_)
    finally:
        dist.destroy_process_group()


def test_dag_row_sharded_world2_matches_one_process(gpu):
    """Node.sample_device(..., group=) with two ranks: every node's rows equal the same rows
    of the one-process evaluation (Sobol and LHS counter-addressed by global row; the reference
    LHS stream decoded whole on each rank; Iman-Conover on Sobol' / reference-stream quantiles
    sharded by column owners (distributed.iman_conover_block), the Cholesky correlator from
    all-reduced statistics, a seeded PermutationCorrelator and a user class run once on rank 0
    and scattered).  An unseeded PermutationCorrelator cannot equal another process's run; its
    ranks' rows together must still be a permutation of each marginal (every rank
    used to climb with its own rng)."""
    import torch.multiprocessing as mp

    from probabilit_amd.distributed import shard_bounds

    n = 1 << 16
    refs = {}
    for kind in _DAG_KINDS:
        root, method = _dag(kind)
        out = root.sample(n, random_state=7, method=method, **_DAG_KW.get(kind, {}))
        if kind == "fund":
            refs[kind] = out
        else:
            refs[kind] = [d.samples_ for d in root.get_parents()]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_dag_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        b = shard_bounds(n, 2)
        for r in range(2):
            np.testing.assert_array_equal(np.load(os.path.join(d, f"fund{r}.npy")), refs["fund"][b[r]:b[r + 1]])
            for kind in _DAG_KINDS[:1] + _DAG_KINDS[2:-1]:
                for j, ref in enumerate(refs[kind]):
                    got = np.load(os.path.join(d, f"{kind}{r}_v{j}.npy"))
                    if kind == "cholesky":
                        # affine in the all-reduced means and Gram matrix, whose sums associate by shard:
                        # an ulp apart (the reference's own BLAS sums agree with either to ~1e-12 only)
                        np.testing.assert_allclose(got, ref[b[r]:b[r + 1]], rtol=1e-13, atol=1e-14)
                    else:
                        np.testing.assert_array_equal(got, ref[b[r]:b[r + 1]])
        for j, ref in enumerate(refs["permcorr_unseeded"]):
            got = np.concatenate([np.load(os.path.join(d, f"permcorr_unseeded{r}_v{j}.npy")) for r in range(2)])
            np.testing.assert_array_equal(np.sort(got), np.sort(ref))


@pytest.mark.parametrize("spec", sorted(SPECS))
def test_world2_on_one_gpu_matches_single_call(gpu, spec):
    import torch.multiprocessing as mp

    from probabilit_amd.distributed import shard_bounds

    ref = _single_call(SPECS[spec])
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), d, spec), nprocs=2, join=True, start_method="spawn")
        parts = [np.load(os.path.join(d, f"y{r}.npy")) for r in range(2)]
    b = shard_bounds(N, 2)
    for r in range(2):
        np.testing.assert_array_equal(parts[r], ref[:, b[r]:b[r + 1]])


def test_rccl_one_rank_forced_collectives(gpu, monkeypatch):
    """The RCCL branch on the box's one GPU: a one-rank "nccl" (RCCL) communicator with
    PBH_FORCE_COLLECTIVES=1 runs every collective of the sharded path for real -- the async
    all-to-alls on the communicator's stream, the side stream that waits for a lane's done
    event, the work handles' waits -- and the result equals the single call."""
    import torch.multiprocessing as mp

    ref = _single_call(SPECS["cfg2"])
    monkeypatch.setenv("PBH_FORCE_COLLECTIVES", "1")
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(1, _free_port(), d, "cfg2", "nccl"), nprocs=1, join=True,
                           start_method="spawn")
        part = np.load(os.path.join(d, "y0.npy"))
    np.testing.assert_array_equal(part, ref)


def test_bench_gpus2_rehearsal_matches_one_gpu(gpu):
    """`bench.py --gpus 2` started without torch.distributed.run launches its two ranks itself
    (here sharing the box's one GPU over gloo), reports n_gpus 2, and each rank's rows of every
    column equal the one-process result on the same seed bit for bit (SHA-1 per column)."""
    import hashlib
    import json
    import subprocess
    import sys

    from probabilit_amd.distributed import shard_bounds

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = 2_000_000
    with tempfile.TemporaryDirectory() as d:
        cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--rows", str(rows), "--steps", "1",
               "--warmup", "0", "--no-cpu", "--no-e2e", "--ppf-rows", "0", "--check-out", d]
        env = dict(os.environ)
        env.pop("WORLD_SIZE", None)
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=root)
        assert r.returncode == 0, r.stderr[-4000:]
        line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        assert line["n_gpus"] == 2 and line["config"]["rows"] == rows
        ranks = [json.load(open(os.path.join(d, f"rank{k}.json"))) for k in range(2)]
    from oracle.pipeline import cfg3_corr, cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    ds = [Distribution(name, **kw) for name, kw in cfg_dists(32)]
    NoOp(*ds).correlate(*ds, corr_mat=cfg3_corr(32)).sample_device(rows, random_state=ranks[0]["seed"], method="lhs")
    b = shard_bounds(rows, 2)
    for k in range(2):
        want = [hashlib.sha1(x.samples_device[b[k]:b[k + 1]].cpu().numpy().tobytes()).hexdigest() for x in ds]
        assert ranks[k]["sha1"] == want, f"rank {k}"
