"""Parity of the headline path at scale (SURVEY.md §8(d) parity gates).

* N = 1e7, d = 32: the bench path itself -- NoOp(*ds).correlate(*ds, C).sample(n,
  method="lhs") on the cfg3 set, i.e. the generated-column fast path (stratum-ordered
  generation, ranks from the LHS permutation, code-bucket step 4, LDS row placement) --
  against the oracle fed the same native quantiles: scipy ppf (oracle.pipeline) and the
  reference's Iman-Conover (oracle.ic, correlation.py:368-425).  Every output value within
  1e-10 relative of the oracle's; at this N adjacent sorted values differ by far more than
  that, so this is also "every step-4 rank identical".
* N = 1e8, d = 32 (the bench size): the §8(d) gate on all 32 columns.  The device's own
  scores S are re-correlated the reference's way (np.corrcoef, cholesky, solve_triangular, then
  @ P.T), ranked as the reference ranks them, and every step-4 index mismatch must be one side
  of an adjacent-rank swap (or exact tie) whose reference |dCS| < 1e-13 (tests/scale_parity.py
  gate_all; tools/parity_1e8.py writes the same document to profiles/).
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


@pytest.mark.timeout(1200)
def test_cfg3_step4_mismatch_gate_1e8_all_columns(gpu):
    """The §8(d) gate at the bench size on all 32 columns (was 4 in round 2): every step-4 index
    the device gets differently from the reference's own order is one side of an adjacent-rank
    swap or an exact tie with reference |dCS| < 1e-13."""
    import json

    import scale_parity as sp

    from oracle.pipeline import cfg3_corr

    doc = sp.gate_all(100_000_000, 32, 0, cfg3_corr(32), threads=16,
                      log=lambda m: print(m if isinstance(m, str) else json.dumps(m), flush=True))
    print(json.dumps({k: v for k, v in doc.items() if k != "columns"}))
    assert doc["violations_total"] == 0, [c for c in doc["columns"] if c["violations"]]
    # the gate's premise: the two CS agree to rounding
    assert doc["max_abs_cs_dev_minus_ref"] < 1e-12, doc["max_abs_cs_dev_minus_ref"]


@pytest.mark.timeout(1200)
def test_cfg3_step4_gate_1e8_reference_steps_1_2(gpu):
    """The same gate with the reference's own steps 1-2: X = scipy ppf of the
    native quantiles (modeling.py:807), S_ref = ndtri(rankdata(X) / (N + 1)) (correlation.py:394-
    395), E_ref = np.corrcoef(S_ref), then cholesky / solve_triangular / @ P.T / rankdata on the
    reference's arrays (:398-422), against the device's production indices on all 32 columns at
    N = 1e8.  Every mismatch must be an adjacent-rank swap or exact tie with reference
    |dCS| < 1e-13; the document (mismatches, their |dCS_ref|, the score and E differences) goes
    to records/ (committed as profiles/r05/parity_1e8_ref_*.json)."""
    import json

    import scale_parity as sp

    from conftest import record
    from oracle.pipeline import cfg3_corr

    doc = sp.gate_all(100_000_000, 32, 0, cfg3_corr(32), threads=16, scores="reference",
                      log=lambda m: print(m if isinstance(m, str) else json.dumps(m), flush=True))
    record("parity_1e8_reference_steps", doc)
    assert all(c["decreases"] == 0 for c in doc["step1"]), doc["step1"]
    assert doc["violations_total"] == 0, [c for c in doc["columns"] if c["violations"]]
    assert doc["max_abs_s_dev_minus_ref"] < 1e-14, doc["max_abs_s_dev_minus_ref"]
    assert doc["max_abs_cs_dev_minus_ref"] < 1e-12, doc["max_abs_cs_dev_minus_ref"]
