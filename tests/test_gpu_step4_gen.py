"""Step 4 of Iman-Conover for generated LHS columns (pbh_step4.hip: MSD code passes, per-bucket
LDS finish emitting (row, sorted position) pairs, row-placement passes, and gen_place
regenerating sort(X)[p] from p) against the oracle's step 4 (correlation.py:418-423) on the
same native quantiles, and against the general path (PBH_STEP4=legacy) bit for bit."""

import numpy as np
import pytest

from conftest import assert_close

pytestmark = pytest.mark.gpu


def _run(n, dists, seed, C, debug_idx=True):
    import ctypes

    from probabilit_amd import _lib, device, qmc
    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.modeling import Distribution

    d = len(dists)
    inst = ImanConover().set_target(C)
    flags = device.zeros(d, "int32")
    cols = []
    for j, (nm, kw) in enumerate(dists):
        v = Distribution(nm, **kw)
        params = [float(p) for p in v._params(n)]
        cols.append(_lib.ICColumn(qmc.seed_from(seed), j, _lib.DIST_IDS[nm], (ctypes.c_double * 4)(*params),
                                  len(params), flags.data_ptr() + 4 * j))
    dbg = {"idx": device.empty((d, n), "int32")} if debug_idx else None
    Y = inst._transform_generated(cols, n, debug=dbg)
    return device.to_host(Y).T, (device.to_host(dbg["idx"]).T if debug_idx else None)


def _oracle(n, dists, seed, C):
    from oracle import ic as oic
    from oracle.pipeline import ppf_columns
    from probabilit_amd import native

    X = ppf_columns(native.fill_lhs(seed, n, len(dists)), dists, threads=8)
    return oic.iman_conover(X, C, threads=8)


@pytest.mark.parametrize("n,d,seed", [(10, 3, 1), (4097, 2, 6), (5000, 8, 2), (300_001, 8, 3), (2**20 + 17, 4, 4),
                                      (4_500_000, 4, 5)])
def test_generated_step4_vs_oracle(gpu, n, d, seed):
    from oracle.pipeline import cfg3_corr, cfg_dists

    dists, C = cfg_dists(d), cfg3_corr(d)
    Y, idx = _run(n, dists, seed, C)
    ref = _oracle(n, dists, seed, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what=f"generated step 4, n={n}")


@pytest.mark.parametrize("n,d,seed", [(70_001, 8, 7), (5_000_000, 3, 8)])
def test_generated_step4_equals_general_path(gpu, monkeypatch, n, d, seed):
    """The regenerating path and the general path (sort(X) read from the workspace, one-sweep
    code sort, value-carrying placement) give the same Y and indices bit for bit."""
    from oracle.pipeline import cfg3_corr, cfg_dists

    dists, C = cfg_dists(d), cfg3_corr(d)
    Y, idx = _run(n, dists, seed, C)
    Y2, _ = _run(n, dists, seed, C, debug_idx=False)
    monkeypatch.setenv("PBH_STEP4", "legacy")
    Yl, idxl = _run(n, dists, seed, C)
    np.testing.assert_array_equal(idx, idxl)
    np.testing.assert_array_equal(Y, Yl)
    np.testing.assert_array_equal(Y2, Y)


@pytest.mark.parametrize("n", [3000, 30_000])
def test_generated_step4_exact_ties(gpu, n):
    """poisson(mu=1e5) in the leading column: its van der Waerden scores tie in small groups
    (each k holds ~2-3 of 3000 draws), so column 0's correlated scores tie exactly and step 4
    takes the 'average' rank of every tie group (idx = int(avg) - 1 shared by the group).  At
    n = 30000 the groups (~25-40 equal codes) exceed the finish's run capacity: the column is
    flagged and redone by the general path."""
    dists = [("poisson", {"mu": 1e5}), ("norm", {}), ("gamma", {"a": 2.0})]
    C = np.array([[1.0, 0.5, 0.2], [0.5, 1.0, 0.3], [0.2, 0.3, 1.0]])
    Y, idx = _run(n, dists, 9, C)
    ref = _oracle(n, dists, 9, C)
    assert len(np.unique(ref["idx"][:, 0])) < n  # the tie groups exist
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what="tie groups")


def test_generated_step4_long_runs_fall_back(gpu):
    """poisson(mu=4) leading: its scores tie in runs of thousands, so the bucket finish flags
    the column (runs longer than 16 equal codes) and it is redone by the general path; the
    result still equals the oracle's."""
    dists = [("poisson", {"mu": 4.0}), ("norm", {}), ("triang", {"c": 0.3})]
    C = np.array([[1.0, 0.4, 0.1], [0.4, 1.0, 0.2], [0.1, 0.2, 1.0]])
    n = 200_000
    Y, idx = _run(n, dists, 3, C)
    ref = _oracle(n, dists, 3, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what="long runs")


@pytest.mark.parametrize("cap", [None, "16"])
def test_generated_step4_run_heads_paths(gpu, monkeypatch, cap):
    """Run heads of a discrete (poisson) column come from the counting pass itself (appended,
    then sorted) when the column has at most PBH_HEADS_CAP distinct values (16384 by default),
    or from the materialised sorted column beyond that (poisson(30) has ~50 distinct values
    in 300 001 draws: the list with the default cap, the fallback with cap 16).  Both give the
    oracle's 'average' ranks and step-4 indices.  (A large mu would reach the fallback with the
    default cap, but scipy's cdflib ppf misses the definition there for ~1 draw in 1e5,
    DESIGN.md section 4, so the oracle's tie groups would differ.)"""
    if cap:
        monkeypatch.setenv("PBH_HEADS_CAP", cap)
    dists = [("poisson", {"mu": 30.0}), ("norm", {}), ("gamma", {"a": 2.0})]
    C = np.array([[1.0, 0.3, 0.2], [0.3, 1.0, 0.4], [0.2, 0.4, 1.0]])
    n = 300_001
    Y, idx = _run(n, dists, 11, C)
    ref = _oracle(n, dists, 11, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what=f"poisson heads, cap={cap}")


def test_generated_step4_two_placement_levels(gpu):
    """2^20 < n <= 2^28: the bucket finish scatters into the top of two row-placement levels and
    one MSD pass resolves the rest; indices and values are the oracle's."""
    from oracle.pipeline import cfg3_corr, cfg_dists

    n, d = 2**21 + 5, 3
    dists, C = cfg_dists(d), cfg3_corr(d)
    Y, idx = _run(n, dists, 12, C)
    ref = _oracle(n, dists, 12, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what="two placement levels")


def test_deferred_tie_check_redoes_the_call(gpu):
    """The tie / inversion checks of continuous generated columns run next to steps 1-3 with
    their scores computed as untied, checked after step 4 (the default PBH_DEFER_COUNTS=3; every
    mode in tests/test_gpu_certificate.py); a column that does tie -- uniform(loc=2**40, scale=1):
    its ulp (2^-12) spans ~24 strata at n = 1e5 -- fails the check and the call is redone with the
    exact counts first, so its 'average' ranks and step-4 indices are the oracle's."""
    dists = [("uniform", {"loc": 2.0**40, "scale": 1.0}), ("norm", {}), ("gamma", {"a": 2.0})]
    C = np.array([[1.0, 0.3, 0.2], [0.3, 1.0, 0.4], [0.2, 0.4, 1.0]])
    n = 100_000
    Y, idx = _run(n, dists, 13, C)
    ref = _oracle(n, dists, 13, C)
    assert len(np.unique(ref["Y"][:, 0])) < n // 10  # the column does tie
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what="deferred tie check")


_VARIANT_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from probabilit_amd import device
from test_gpu_step4_gen import _debug_run
out = _debug_run({n}, {dists!r}, {seed}, np.array({C!r}))
for k, v in out.items():
    np.save({d!r} + "/" + k + ".npy", v)
"""


def _debug_run(n, dists, seed, C):
    """Y, idx, S and E of the generated-column path (debug outputs of pbh_iman_conover)."""
    import ctypes

    from probabilit_amd import _lib, device, qmc
    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.modeling import Distribution

    d = len(dists)
    inst = ImanConover().set_target(C)
    flags = device.zeros(d, "int32")
    cols = []
    for j, (nm, kw) in enumerate(dists):
        v = Distribution(nm, **kw)
        params = [float(p) for p in v._params(n)]
        cols.append(_lib.ICColumn(qmc.seed_from(seed), j, _lib.DIST_IDS[nm], (ctypes.c_double * 4)(*params),
                                  len(params), flags.data_ptr() + 4 * j))
    dbg = {"idx": device.empty((d, n), "int32"), "S": device.empty((d, n), "float64"), "E": np.zeros((d, d))}
    Y = inst._transform_generated(cols, n, debug=dbg)
    return {"Y": device.to_host(Y).T, "idx": device.to_host(dbg["idx"]).T, "S": device.to_host(dbg["S"]).T,
            "E": dbg["E"].copy()}


@pytest.mark.timeout(900)
def test_step4_variants_match_the_oracle(gpu, tmp_path):
    """Every A/B switch of the generated-column path, each in its own process (they are read
    once): 4096-row code-pass tiles (PBH_MSD_TILE=4096), the whole gamma table in LDS
    (PBH_GAMMA_WIN=0), the placement levels' other split (PBH_PLACE_TOP=0), 64-row step-3 tiles
    (PBH_APPLY_ROWS=64), the poisson run heads from every stratum instead of the boundary search
    (PBH_DISCRETE_SCAN=1), the code histogram with the tile-class counts per code (PBH_HIST_CLASS=0),
    step 3 with one-row accesses (PBH_APPLY_W2=0; the default pairs rows in 16-byte accesses, the odd
    N taking its one-row tail) or with cached paired accesses (PBH_APPLY_NT=0; the default is non-temporal),
    the discrete columns' values through the inverse CDF per row (PBH_PLACE_RUNS=0; the default reads
    them from the run table) -- step-4 indices equal to the oracle's and the outputs within 1e-10.  600 001 rows: 8 histogram
    blocks per column, so the default takes the class-major k_hist16c."""
    import os
    import subprocess
    import sys

    from oracle.pipeline import cfg3_corr, cfg_dists

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n, d, seed = 600_001, 8, 31
    dists, C = cfg_dists(d), cfg3_corr(d)
    ref = _oracle(n, dists, seed, C)
    for env in ({"PBH_HIST_CLASS": "0"}, {"PBH_MSD_TILE": "4096"}, {"PBH_GAMMA_WIN": "0"}, {"PBH_PLACE_TOP": "0"},
                {"PBH_APPLY_ROWS": "64"},
                {"PBH_DISCRETE_SCAN": "1"}, {"PBH_APPLY_W2": "0"}, {"PBH_APPLY_NT": "0"}, {"PBH_PLACE_RUNS": "0"}):
        dd = tmp_path / "_".join(f"{k}{v}" for k, v in env.items())
        dd.mkdir()
        script = _VARIANT_SCRIPT.format(root=root, tests=os.path.join(root, "tests"), d=str(dd), n=n, dists=dists,
                                      seed=seed, C=C.tolist())
        r = subprocess.run([sys.executable, "-c", script], env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, (env, r.stderr[-3000:])
        np.testing.assert_array_equal(np.load(dd / "idx.npy"), ref["idx"], err_msg=str(env))
        assert_close(np.load(dd / "Y.npy"), ref["Y"], rtol=1e-10, what=str(env))


@pytest.mark.parametrize("dists", [[("norm", {}), ("poisson", {"mu": 2000.0}), ("binom", {"n": 50, "p": 0.4})],
                                   [("gamma", {"a": 2.0}), ("bernoulli", {"p": 0.3}), ("poisson", {"mu": 0.5})]])
def test_discrete_placement_from_runs(gpu, dists):
    """A discrete column's step-4 values come from its run table (k_place_gen_runs: the value of
    each run of equal strata values, found through a guide over the stratum) instead of the
    inverse CDF of every row: poisson(2000) has ~400 runs, many of them shorter than a guide cell
    in the tails; bernoulli two; binom and poisson(0.5) a handful.  Indices and values are the
    oracle's."""
    C = np.array([[1.0, 0.5, 0.2], [0.5, 1.0, 0.3], [0.2, 0.3, 1.0]])
    n = 300_001
    Y, idx = _run(n, dists, 17, C)
    ref = _oracle(n, dists, 17, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what=f"runs placement {dists}")


@pytest.mark.parametrize("shape", [0.1, 0.25])
def test_gamma_placement_slow_list(gpu, shape):
    """Small gamma shapes leave guide intervals without the midpoint check (coverage is complete
    only for a >= 0.3), so the step-4 placement sends many items to the slow list that
    k_place_gen_gamma_slow evaluates after the windowed kernel (with a = 0.1 more than the list
    holds at this N: the second kernel then evaluates every row).  Indices and values equal the
    oracle's."""
    dists = [("gamma", {"a": shape}), ("norm", {}), ("gamma", {"a": shape, "scale": 2.0})]
    C = np.array([[1.0, 0.4, 0.2], [0.4, 1.0, 0.3], [0.2, 0.3, 1.0]])
    Y, idx = _run(200_003, dists, 41, C)
    ref = _oracle(200_003, dists, 41, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what=f"gamma(a={shape}) placement")


def test_bad_last_column_returns_an_error_and_leaves_the_device_usable(gpu):
    """A column list whose LAST entry has a bad parameter count: pbh_iman_conover has by then
    queued the earlier columns' tables and counts on the step-4 side streams, so its error return
    must join those streams before their tables are freed.  The call raises, and the
    same columns with the count fixed then give the oracle's result."""
    import ctypes

    from probabilit_amd import _lib, device, qmc
    from probabilit_amd.correlation import ImanConover
    from probabilit_amd.modeling import Distribution

    dists = [("poisson", {"mu": 4.0}), ("gamma", {"a": 2.0}), ("norm", {}), ("poisson", {"mu": 30.0})]
    C = np.array([[1.0, 0.4, 0.2, 0.1], [0.4, 1.0, 0.3, 0.2], [0.2, 0.3, 1.0, 0.3], [0.1, 0.2, 0.3, 1.0]])
    n = 200_001
    flags = device.zeros(len(dists), "int32")
    cols = []
    for j, (nm, kw) in enumerate(dists):
        params = [float(p) for p in Distribution(nm, **kw)._params(n)]
        cols.append(_lib.ICColumn(qmc.seed_from(5), j, _lib.DIST_IDS[nm], (ctypes.c_double * 4)(*params),
                                  len(params) + (1 if j == len(dists) - 1 else 0), flags.data_ptr() + 4 * j))
    with pytest.raises(Exception):
        ImanConover().set_target(C)._transform_generated(cols, n)
    device.synchronize()
    Y, idx = _run(n, dists, 5, C)
    ref = _oracle(n, dists, 5, C)
    np.testing.assert_array_equal(idx, ref["idx"])
    assert_close(Y, ref["Y"], rtol=1e-10, what="after the failed call")
