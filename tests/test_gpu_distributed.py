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

SPEC = [(0, [0.0, 1.0]), (5, [2.0, 0.0, 1.0]), (4, [0.3, 0.0, 1.0]), (6, [4.0, 0.0]), (0, [5.0, 2.0]),
        (5, [0.7, 0.0, 3.0]), (4, [0.8, 1.0, 2.0]), (6, [30.0, 0.0])]
N = 300_007
SEED = 12345


def _target():
    from oracle.pipeline import cfg3_corr

    return cfg3_corr(len(SPEC))


def _single_call():
    from probabilit_amd import _lib, device
    from probabilit_amd.correlation import ImanConover

    flags = device.zeros(len(SPEC), "int32")
    cols = [_lib.ICColumn(SEED, c, d, (ctypes.c_double * 3)(*p), len(p), flags.data_ptr() + 4 * c)
            for c, (d, p) in enumerate(SPEC)]
    Y = ImanConover().set_target(_target())._transform_generated(cols, N)
    return device.to_host(Y)


def _columns():
    from probabilit_amd.distributed import LHSColumn

    return [LHSColumn(SEED, c, d, p) for c, (d, p) in enumerate(SPEC)]


def test_world1_matches_single_call(gpu):
    from probabilit_amd import device
    from probabilit_amd.distributed import iman_conover_lhs

    ref = _single_call()
    Y = iman_conover_lhs(_columns(), np.linalg.cholesky(_target()), N)
    np.testing.assert_array_equal(device.to_host(Y), ref)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from probabilit_amd import device
        from probabilit_amd.distributed import iman_conover_lhs

        Y = iman_conover_lhs(_columns(), np.linalg.cholesky(_target()), N)
        np.save(os.path.join(outdir, f"y{rank}.npy"), device.to_host(Y))
    finally:
        dist.destroy_process_group()


def _dag(kind):
    from oracle.pipeline import cfg_dists
    from probabilit_amd.modeling import Distribution, NoOp

    if kind == "correlated":
        ds = [Distribution(name, **kw) for name, kw in cfg_dists(8)]
        return NoOp(*ds).correlate(*ds, corr_mat=_target()), "lhs"
    r = 0
    for _ in range(20):  # README mutual-fund loop (BASELINE config 5)
        r = r * Distribution("norm", loc=1.11, scale=0.15) + 1200
    return r, "sobol"


def _dag_worker(rank, world, port, outdir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from probabilit_amd import device

        for kind in ("correlated", "fund"):
            root, method = _dag(kind)
            out = root.sample_device(1 << 16, random_state=7, method=method, group=dist.group.WORLD)
            if kind == "fund":
                np.save(os.path.join(outdir, f"{kind}{rank}.npy"), device.to_host(out))
            else:
                for j, d in enumerate(root.get_parents()):
                    np.save(os.path.join(outdir, f"{kind}{rank}_v{j}.npy"), d.samples_)
    finally:
        dist.destroy_process_group()


def test_dag_row_sharded_world2_matches_one_process(gpu):
    """Node.sample_device(..., group=) with two ranks: every node's rows equal the same rows
    of the one-process evaluation (Sobol and LHS counter-addressed by global row)."""
    import torch.multiprocessing as mp

    from probabilit_amd.distributed import shard_bounds

    n = 1 << 16
    refs = {}
    for kind in ("correlated", "fund"):
        root, method = _dag(kind)
        out = root.sample(n, random_state=7, method=method)
        if kind == "fund":
            refs[kind] = out
        else:
            refs["vars"] = [d.samples_ for d in root.get_parents()]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_dag_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        b = shard_bounds(n, 2)
        for r in range(2):
            np.testing.assert_array_equal(np.load(os.path.join(d, f"fund{r}.npy")), refs["fund"][b[r]:b[r + 1]])
            for j, ref in enumerate(refs["vars"]):
                np.testing.assert_array_equal(np.load(os.path.join(d, f"correlated{r}_v{j}.npy")), ref[b[r]:b[r + 1]])


def test_world2_on_one_gpu_matches_single_call(gpu):
    import torch.multiprocessing as mp

    from probabilit_amd.distributed import shard_bounds

    ref = _single_call()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        parts = [np.load(os.path.join(d, f"y{r}.npy")) for r in range(2)]
    b = shard_bounds(N, 2)
    for r in range(2):
        np.testing.assert_array_equal(parts[r], ref[:, b[r]:b[r + 1]])
