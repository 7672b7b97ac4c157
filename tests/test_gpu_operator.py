"""The operator API at the sizes where step 1 takes its large-n path (n >= 2^22): the column sorted
on its top 48 key bits with the runs of equal top bits ordered by a fix-up (a run longer than the
fix-up takes sends the column back to the full sort), the scores written in rank order and put in
row order by the row placement, X and Y transposed once.  Against the oracle and against the
comparator paths (PBH_SCORES_PLACE=0: every byte sorted, the scores scattered; PBH_IC_TRANSPOSE=0:
strided columns), bit for bit."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _design(n):
    rng = np.random.default_rng(21)
    x0 = rng.normal(size=n)
    x1 = rng.gamma(2.0, size=n)
    # a long run of values equal in their top 48 key bits but not in the low 16: the redo path
    x1[1000:1300] = 1.0 + np.arange(300) * 2.0**-52
    x2 = rng.uniform(size=n)
    # short runs (pairs / triples) of equal top 48 bits with different low bits: the fix-up
    idx = rng.choice(n, 3000, replace=False)
    x2[idx[:1000]] = x2[idx[1000:2000]] + 2.0**-50
    x2[idx[2000:]] = x2[idx[1000:2000]] - 2.0**-51
    x3 = rng.poisson(4.0, size=n).astype(float)  # integers: the low bytes constant, nothing to fix
    return np.column_stack([x0, x1, x2, x3])


def test_operator_large_n_paths_bit_exact(gpu):
    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd.correlation import ImanConover

    n = (1 << 22) + 3
    X = _design(n)
    C = cfg3_corr(4)
    Y = ImanConover().set_target(C)(X)
    np.testing.assert_array_equal(Y, oic.iman_conover(X, C)["Y"])
    # the switches are read once per process: the comparators run in a child each
    import subprocess
    import sys

    code = (
        "import os, sys, numpy as np; sys.path.insert(0, os.getcwd()); sys.path.insert(0, 'tests');"
        "from test_gpu_operator import _design; from oracle.pipeline import cfg3_corr;"
        "from probabilit_amd.correlation import ImanConover;"
        f"X = _design({n}); Y = ImanConover().set_target(cfg3_corr(4))(X); np.save(sys.argv[1], Y)"
    )
    import os
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "y.npy")
        for env in ({"PBH_SCORES_PLACE": "0"}, {"PBH_IC_TRANSPOSE": "0"}):
            p = subprocess.run([sys.executable, "-c", code, out], env=dict(os.environ, **env), capture_output=True,
                               text=True, timeout=600, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
            assert p.returncode == 0, p.stderr[-2000:]
            np.testing.assert_array_equal(np.load(out), Y)


def test_column_scores_large_n(gpu):
    """pbh_ic_column_scores (the row-sharded operator's step 1 on an owned column) at n >= 2^22:
    the scores within the van der Waerden gate of the oracle's (ndtri of rankdata / (n + 1)), the
    sorted column exact, for the same columns (a run that takes the redo, short runs, integers)."""
    import torch

    from oracle import ic as oic
    from oracle.pipeline import cfg3_corr
    from probabilit_amd import device
    from probabilit_amd.distributed import HipPhases

    n = (1 << 22) + 3
    X = _design(n)
    ref = oic.iman_conover(X, cfg3_corr(4))["S"]
    ph = HipPhases()
    for c in range(X.shape[1]):
        x = device.to_device(np.ascontiguousarray(X[:, c]))
        s = torch.empty_like(x)
        sx = torch.empty_like(x)
        flag = torch.zeros(1, dtype=torch.int32, device=x.device)
        ph.column_scores(x, s, sx, flag)
        np.testing.assert_array_equal(device.to_host(sx), np.sort(X[:, c]))
        np.testing.assert_allclose(device.to_host(s), ref[:, c], rtol=0, atol=1e-14)
        assert int(flag.item()) == 0
