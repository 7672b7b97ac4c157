"""Parity of the headline path at scale (SURVEY.md §8(d) parity gates).

* N = 1e7, d = 32: the bench path itself -- NoOp(*ds).correlate(*ds, C).sample(n,
  method="lhs") on the cfg3 set, i.e. the generated-column fast path (stratum-ordered
  generation, ranks from the LHS permutation, code-bucket step 4, LDS row placement) --
  against the oracle fed the same native quantiles: scipy ppf (oracle.pipeline) and the
  reference's Iman-Conover (oracle.ic, correlation.py:368-425).  Every output value within
  1e-10 relative of the oracle's; at this N adjacent sorted values differ by far more than
  that, so this is also "every step-4 rank identical".
* N = 1e8, d = 32 (the bench size): the §8(d) gate.  The device's own scores S are
  re-correlated the reference's way (cholesky, solve_triangular, then @ P.T) for the first
  four columns (they depend on the first four score columns only), ranked as the reference
  ranks them, and every step-4 index mismatch must be one side of an adjacent-rank swap whose
  reference |dCS| < 1e-13.  tools/parity_1e8.py does all 32 columns with E recomputed by
  np.corrcoef (profiles/r02/parity_1e8.json).
"""

import numpy as np
import pytest

from conftest import assert_close

pytestmark = pytest.mark.gpu

THREADS = 16  # the GPU box's CPU share per GPU


@pytest.mark.timeout(600)
def test_cfg3_bench_path_vs_oracle_1e7(gpu):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr, cfg_dists, ppf_columns
    from probabilit_amd import device, native
    from probabilit_amd.modeling import Distribution, NoOp

    n, d, seed = 10_000_000, 32, 5
    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    C = cfg3_corr(d)
    NoOp(*ds).correlate(*ds, corr_mat=C).sample_device(n, random_state=seed, method="lhs")
    Y = np.empty((n, d))
    for j, x in enumerate(ds):
        Y[:, j] = device.to_host(x.samples_device)
    Q = native.fill_lhs(seed, n, d)  # the native quantile matrix of this seed (row order)
    X = ppf_columns(Q, cfg_dists(d), threads=THREADS)
    del Q
    ref = oic.iman_conover(X, C, threads=THREADS)
    Yr = ref["Y"]
    mism = int(np.count_nonzero(np.abs(Y - Yr) > 1e-10 * np.abs(Yr)))
    assert mism == 0, f"{mism} of {Y.size} outputs differ from the oracle by more than 1e-10 relative"
    assert_close(Y, Yr, rtol=1e-10, what="cfg3 N=1e7 bench path vs oracle")


@pytest.mark.timeout(900)
def test_cfg3_step4_mismatch_gate_1e8(gpu):
    import scale_parity as sp

    from oracle.pipeline import cfg3_corr
    from probabilit_amd import device

    n, d, seed, k = 100_000_000, 32, 0, 4
    Y, S, CS, E, P, gen = sp.run_device(n, d, seed, cfg3_corr(d))
    S4 = device.to_host(S[:k])
    y4 = [device.to_host(Y[j]) for j in range(k)]
    cs4 = [device.to_host(CS[j]) for j in range(k)]
    del Y, S, CS
    sx4 = [sp.sorted_x(gen[j], n) for j in range(k)]
    cs_ref = sp.reference_cs(S4, E, P, k=k)
    res = sp.gate(cs_ref, y4, sx4, cs4, threads=k)
    for r in res:
        print(r)
        assert r["violations"] == 0, r
    # the gate's premise: the two CS agree to rounding
    worst = max(float(np.max(np.abs(cs4[j] - cs_ref[:, j]))) for j in range(k))
    assert worst < 1e-12, worst
