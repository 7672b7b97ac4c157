"""Row-sharded Iman-Conover (probabilit_amd/distributed.py) under the gloo
backend with world sizes 1 to 4 on CPU (uneven row shards, ranks owning 2, 1 or no column): the exchange logic (run-head all-gather, sum and
Gram all-reduces, the two all-to-alls) with numpy phases (tests/dist_cpu_phases.py), against
the oracle's single-process ImanConover on the same LHS design.  The GPU phases of the same
orchestrator are checked in test_gpu_distributed.py."""

import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.ic import iman_conover
from oracle.pipeline import cfg3_corr

CASES = {
    # (n, [(dist id, params)]): continuous + tied (poisson) columns, uneven shards
    "mixed": (3001, [(0, [0.0, 1.0]), (6, [4.0, 0.0]), (5, [2.0, 0.0, 1.0]), (4, [0.3, 0.0, 1.0]),
                     (6, [30.0, 0.0])]),
    "two": (2048, [(0, [5.0, 2.0]), (5, [0.7, 0.0, 3.0])]),
    # lognorm(s=1000) overflows to inf above q ~ 0.76 (and to 0 below ~ 0.23): flag bit 0
    "nonfinite": (2001, [(0, [0.0, 1.0]), (3, [1000.0, 0.0, 1.0]), (5, [2.0, 0.0, 1.0])]),
}
EXPECTED_FLAGS = {"mixed": [0, 0, 0, 0, 0], "two": [0, 0], "nonfinite": [0, 1, 0]}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _columns(spec):
    from probabilit_amd.distributed import LHSColumn

    return [LHSColumn(0, c, d, p) for c, (d, p) in enumerate(spec)]


def _worker(rank, world, port, case, outdir, redo=(), defer=False):
    import torch
    import torch.distributed as dist

    from dist_cpu_phases import CpuPhases, design
    from probabilit_amd.distributed import iman_conover_lhs

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n, spec = CASES[case]
        perms, us = design(n, len(spec), seed=3)
        P = np.linalg.cholesky(cfg3_corr(len(spec)))
        flags = torch.zeros(len(spec), dtype=torch.int32)
        # with defer, rank 0's first count of column 0 (continuous in every case) reports a false
        # tie: the deferred check must redo the whole call on every rank
        ph = CpuPhases(perms, us, redo=redo if rank == 0 else (), fake_tie=0 if (defer and rank == 0) else None)
        Y = iman_conover_lhs(_columns(spec), P, n, phases=ph, flags=flags, defer=defer)
        np.save(os.path.join(outdir, f"y{rank}.npy"), Y.numpy())
        np.save(os.path.join(outdir, f"f{rank}.npy"), flags.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,redo,defer", [(1, (), False), (2, (), False), (3, (), False), (4, (), False),
                                              (2, (0,), False), (3, (1,), False), (1, (), True), (3, (), True)])
@pytest.mark.parametrize("case", sorted(CASES))
def test_sharded_ic_matches_single_process_oracle(world, redo, defer, case):
    """redo: rank 0 "rejects" its owned column index `redo` on the fast path (garbage positions
    leave first, the general path's after finish): the re-send must repair every rank's rows.
    defer: the continuous columns' counts run after step 3; rank 0 reports a false tie in the
    deferred count, so every rank must redo the call with the counts first."""
    from dist_cpu_phases import column_values, design
    from probabilit_amd.distributed import shard_bounds

    n, spec = CASES[case]
    perms, us = design(n, len(spec), seed=3)
    cols = _columns(spec)
    X = np.column_stack([column_values(c, perms, us, n) for c in cols])
    ref = iman_conover(X, cfg3_corr(len(spec)))["Y"]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), case, d, redo, defer), nprocs=world, join=True,
                           start_method="spawn")
        parts = [np.load(os.path.join(d, f"y{r}.npy")) for r in range(world)]
        flags = [np.load(os.path.join(d, f"f{r}.npy")).tolist() for r in range(world)]
    # flag words are OR-combined across ranks (bits unchanged), identical on every rank
    assert flags == [EXPECTED_FLAGS[case]] * world
    b = shard_bounds(n, world)
    for r, part in enumerate(parts):
        assert part.shape == (len(spec), b[r + 1] - b[r])
        np.testing.assert_array_equal(part.T, ref[b[r]:b[r + 1]])


def test_shard_bounds_cover_rows():
    from probabilit_amd.distributed import shard_bounds

    for n in (1, 7, 4096, 100_000_001):
        for w in (1, 2, 3, 8):
            b = shard_bounds(n, w)
            assert b[0] == 0 and b[-1] == n and all(b[i] <= b[i + 1] for i in range(w))


# ---- materialised blocks (Sobol' / Halton / MT / reference-stream quantiles, composite params):
# distributed.iman_conover_block ranks each column on its owner, no rank holds the whole block
def _block_case(n, seed=5):
    rng = np.random.default_rng(seed)
    X = np.column_stack([rng.normal(size=n), rng.poisson(4.0, size=n).astype(float), rng.gamma(2.0, size=n),
                         rng.poisson(30.0, size=n).astype(float), rng.uniform(size=n)])
    return X


def _block_worker(rank, world, port, n, outdir):
    import torch
    import torch.distributed as dist

    from dist_cpu_phases import CpuPhases
    from probabilit_amd import distributed as D

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X = _block_case(n)
        b = D.shard_bounds(n, world)
        block = torch.from_numpy(np.ascontiguousarray(X[b[rank]:b[rank + 1]].T))
        P = np.linalg.cholesky(cfg3_corr(X.shape[1]))
        Y = D.iman_conover_block(block, P, n, phases=CpuPhases([], []))
        np.save(os.path.join(outdir, f"y{rank}.npy"), Y.numpy())
        mean, gram = D.block_stats(block, n, phases=CpuPhases([], []))
        np.save(os.path.join(outdir, f"m{rank}.npy"), mean)
        np.save(os.path.join(outdir, f"g{rank}.npy"), gram)
        full = D.gather_to_root(block, n, dist.group.WORLD)
        if rank == 0:
            np.save(os.path.join(outdir, "full.npy"), full.numpy())
            full = full * 2.0
        back = D.scatter_from_root(full, X.shape[1], n, dist.group.WORLD, like=block)
        np.save(os.path.join(outdir, f"b{rank}.npy"), back.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_block_ic_matches_single_process_oracle(world):
    """Iman-Conover on a row-sharded materialised block (continuous and tied columns, uneven
    shards, ranks owning 2, 1 or no column): every rank's rows equal the oracle's single-process
    result; the Cholesky statistics equal numpy's; the root gather / scatter round trip."""
    from probabilit_amd.distributed import shard_bounds

    n = 2999
    X = _block_case(n)
    ref = iman_conover(X, cfg3_corr(X.shape[1]))["Y"]
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_block_worker, args=(world, _free_port(), n, d), nprocs=world, join=True,
                           start_method="spawn")
        b = shard_bounds(n, world)
        for r in range(world):
            np.testing.assert_array_equal(np.load(os.path.join(d, f"y{r}.npy")).T, ref[b[r]:b[r + 1]])
            np.testing.assert_allclose(np.load(os.path.join(d, f"m{r}.npy")), X.mean(axis=0), rtol=1e-13)
            D = X - X.mean(axis=0)
            np.testing.assert_allclose(np.load(os.path.join(d, f"g{r}.npy")), D.T @ D, rtol=1e-11)
            np.testing.assert_array_equal(np.load(os.path.join(d, f"b{r}.npy")).T, 2.0 * X[b[r]:b[r + 1]])
        np.testing.assert_array_equal(np.load(os.path.join(d, "full.npy")).T, X)
