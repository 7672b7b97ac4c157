"""The tie / inversion certificate of the deferred step-1 check (k_cert_scan / k_cert_eval,
pbh_ppf.hip; pbh_lhs_sorted_counts(certify=1)) against the exact counts (k_lhs_sorted_ppf), and
every PBH_DEFER_COUNTS mode end to end (modes 0-2 had no GPU coverage).

The certificate may only answer "no tie, no inversion"; anything it cannot certify reads as a
count, which makes the caller recount exactly."""

import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _counts(name, kw, n, t0, nt, certify, col=0, seed=7):
    from probabilit_amd import _lib, device
    from probabilit_amd.modeling import _parse_scipy_args

    params = [float(v) for v in _parse_scipy_args(name, (), kw)]
    counts, flag = device.zeros(2, "int64"), device.zeros(1, "int32")
    lib = _lib.load()
    _lib.check(lib.pbh_lhs_sorted_counts(seed, n, t0, nt, col, _lib.DIST_IDS[name], (ctypes.c_double * 3)(*params),
                                         len(params), counts.data_ptr(), None, None, 0, flag.data_ptr(), int(certify),
                                         device.stream()))
    return device.to_host(counts).tolist(), int(device.to_host(flag)[0])


CONTINUOUS = [("norm", {}), ("norm", {"loc": 5.0, "scale": 2.0}), ("gamma", {"a": 2.0}),
              ("gamma", {"a": 0.7, "scale": 3.0}), ("triang", {"c": 0.3}), ("triang", {"c": 0.8, "loc": 1.0, "scale": 2.0}),
              ("uniform", {}), ("expon", {"scale": 0.5}), ("lognorm", {"s": 0.4, "scale": 1.5})]


@pytest.mark.parametrize("name,kw", CONTINUOUS)
def test_certificate_agrees_with_exact_counts(gpu, name, kw):
    """cfg2/cfg3's continuous families (and the others of the fused LHS path) at N = 1e8, the
    whole column and a shard's segment (t0 = row0 - 1): certified, as the exact counts say."""
    n = 100_000_000
    for t0, nt in ((0, n), (n // 3 - 1, n // 3 + 1)):
        exact, f0 = _counts(name, kw, n, t0, nt, certify=False)
        cert, f1 = _counts(name, kw, n, t0, nt, certify=True)
        assert exact == [0, 0] and f0 == 0, (name, kw, exact)
        assert cert == [0, 0] and f1 == 0, (name, kw, cert)


def test_certificate_never_certifies_a_tie(gpu, monkeypatch):
    """uniform(loc=2^40): its ulp spans ~24 strata at n = 1e5, so the column ties.  Its bound
    makes the certificate decline (the exact counts run, finding the ties); forcing every pair
    to be a candidate (PBH_CERT_T=1) evaluates them all, and the certificate's counts then equal
    the exact ones.  lognorm(s=1000) overflows to inf: a non-finite end is flagged and reported."""
    n = 100_000
    exact, _ = _counts("uniform", {"loc": 2.0**40}, n, 0, n, certify=False)
    assert exact[0] > 0
    assert _counts("uniform", {"loc": 2.0**40}, n, 0, n, certify=True)[0] == exact
    monkeypatch.setenv("PBH_CERT_T", "1")
    assert _counts("uniform", {"loc": 2.0**40}, n, 0, n, certify=True)[0] == exact
    monkeypatch.delenv("PBH_CERT_T")
    cert, flag = _counts("lognorm", {"s": 1000.0}, 2000, 0, 2000, certify=True)
    assert flag == 1 and cert[0] > 0


_SCRIPT = r"""
import json, sys
import numpy as np
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
from test_gpu_step4_gen import _run
C = np.array([[1.0, 0.3, 0.2], [0.3, 1.0, 0.4], [0.2, 0.4, 1.0]])
out = {{}}
for tag, dists in (("ties", [("uniform", {{"loc": 2.0**40, "scale": 1.0}}), ("norm", {{}}), ("gamma", {{"a": 2.0}})]),
                   ("plain", [("norm", {{}}), ("poisson", {{"mu": 4.0}}), ("triang", {{"c": 0.3}})])):
    Y, idx = _run(100_000, dists, 13, C)
    np.save({d!r} + "/" + tag + "_y.npy", Y); np.save({d!r} + "/" + tag + "_i.npy", idx)
"""


@pytest.mark.timeout(600)
def test_every_deferral_mode_matches_the_oracle(gpu, tmp_path):
    """PBH_DEFER_COUNTS 0 (counts first), 1 (next to steps 1-3, checked before step 4), 2 (next
    to step 4), 3 (default: next to steps 1-3, checked at the end), and 3 with the exact counts
    instead of the certificate (PBH_CERT=0), each in its own process (the mode is read once): a
    column that ties (uniform(loc=2^40)) redoes the call, a column set that does not, all equal
    to the oracle."""
    from test_gpu_step4_gen import _oracle

    from conftest import assert_close

    C = np.array([[1.0, 0.3, 0.2], [0.3, 1.0, 0.4], [0.2, 0.4, 1.0]])
    refs = {"ties": _oracle(100_000, [("uniform", {"loc": 2.0**40, "scale": 1.0}), ("norm", {}), ("gamma", {"a": 2.0})],
                            13, C),
            "plain": _oracle(100_000, [("norm", {}), ("poisson", {"mu": 4.0}), ("triang", {"c": 0.3})], 13, C)}
    for env in ({"PBH_DEFER_COUNTS": "0"}, {"PBH_DEFER_COUNTS": "1"}, {"PBH_DEFER_COUNTS": "2"},
                {"PBH_DEFER_COUNTS": "3"}, {"PBH_DEFER_COUNTS": "3", "PBH_CERT": "0"}):
        d = tmp_path / "_".join(f"{k}{v}" for k, v in env.items())
        d.mkdir()
        script = _SCRIPT.format(root=ROOT, tests=os.path.join(ROOT, "tests"), d=str(d))
        r = subprocess.run([sys.executable, "-c", script], env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, (env, r.stderr[-3000:])
        for tag, ref in refs.items():
            np.testing.assert_array_equal(np.load(d / f"{tag}_i.npy"), ref["idx"], err_msg=json.dumps(env))
            assert_close(np.load(d / f"{tag}_y.npy"), ref["Y"], rtol=1e-10, what=f"{env} {tag}")


_HEADS_SCRIPT = r"""
import ctypes, json, sys
import numpy as np
sys.path.insert(0, {root!r})
from probabilit_amd import _lib, device
out = {{}}
lib = _lib.load()
for mu, n, t0, nt in {cases!r}:
    counts, flag = device.zeros(2, "int64"), device.zeros(1, "int32")
    heads, hcur = device.zeros(16384, "int32"), device.zeros(1, "int32")
    _lib.check(lib.pbh_lhs_sorted_counts(11, n, t0, nt, 3, _lib.DIST_IDS["poisson"], (ctypes.c_double * 3)(mu, 0.0, 0.0),
                                         2, counts.data_ptr(), heads.data_ptr(), hcur.data_ptr(), 16384, flag.data_ptr(),
                                         0, device.stream()))
    h = int(device.to_host(hcur)[0])
    out[f"{{mu}}_{{n}}_{{t0}}"] = {{"counts": device.to_host(counts).tolist(), "flag": int(device.to_host(flag)[0]),
                                   "heads": sorted(device.to_host(heads)[:min(h, 16384)].tolist()), "hcur": h}}
print(json.dumps(out))
"""


@pytest.mark.timeout(300)
def test_poisson_boundary_search_equals_the_scan(gpu):
    """A poisson column's tie count and run heads from the boundary search (k_discrete_heads: one
    binary search per distinct value) equal the stratum-by-stratum scan's (PBH_DISCRETE_SCAN=1,
    its own process) exactly: whole columns and shard segments (t0 = row0 - 1), mu 4 / 30 / 400."""
    cases = [(4.0, 10_000_000, 0, 10_000_000), (30.0, 10_000_000, 0, 10_000_000), (400.0, 3_000_001, 0, 3_000_001),
             (30.0, 10_000_000, 3_333_332, 3_333_334), (4.0, 1000, 0, 1000), (400.0, 50, 0, 50)]
    res = []
    for env in ({}, {"PBH_DISCRETE_SCAN": "1"}):
        r = subprocess.run([sys.executable, "-c", _HEADS_SCRIPT.format(root=ROOT, cases=cases)],
                           env={**os.environ, **env}, capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, (env, r.stderr[-3000:])
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1]
    for k, v in res[0].items():
        assert v["counts"][1] == 0 and v["flag"] == 0, (k, v)
