"""Values, not only ranks, at the BASELINE sizes (SURVEY.md §8(d) gates).

* cfg3, N = 1e8: every column's stratum-ordered values -- the inputs step 1 counts and step 4
  regenerates as sort(X)[p] -- on 10^6 random strata against scipy.stats.<dist>.ppf of the same
  native quantiles (1e-10 relative; poisson exact).
* cfg3, N = 1e8, poisson columns: every one of the 1e8 strata near a CDF boundary (relative
  window 1e-6 around each pdtr(k, mu), 10^4 times scipy's widest deviation from the definition at
  these mu) against scipy; between boundaries both are constant in q, so this compares every
  output of the column.  They must be equal (the device runs scipy's pdtrik search inside the
  windows, pbh_cdflib.h); the counts, including how often scipy differs from the definition
  there, go to records/.
* cfg2, N = 1e7, d = 8, uncorrelated, through Node.sample_device: against oracle.pipeline's scipy
  ppf of the same native quantile matrix.
* cfg5, N = 1e8 (Sobol', seed 3: a seed whose points avoid q = 0): the fused graph kernel's sink
  equals the per-node path's bit for bit, and a block of 10^6 rows equals the oracle's mutual fund
  (scipy ppf + numpy arithmetic on the same Sobol' points).
"""

import ctypes

import numpy as np
import pytest

from conftest import assert_close, record

pytestmark = pytest.mark.gpu

THREADS = 16
N8 = 100_000_000
RTOL = 1e-10


def _sorted_columns(seed, n, col, name, kw):
    """(device sorted values, device sorted quantiles) of native-LHS column `col`: the
    stratum-ordered generator's values (pbh_lhs_sorted_ppf, what step 1 counts and step 4
    regenerates) and the quantile of every stratum (the sorted pbh_fill_lhs column)."""
    import torch

    from probabilit_amd import _lib, device
    from probabilit_amd.modeling import _parse_scipy_args

    params = [float(v) for v in _parse_scipy_args(name, (), kw)]
    out, flag = device.empty(n), device.zeros(1, "int32")
    lib = _lib.load()
    _lib.check(lib.pbh_lhs_sorted_ppf(seed, n, 0, n, col, _lib.DIST_IDS[name], (ctypes.c_double * 3)(*params),
                                      len(params), out.data_ptr(), flag.data_ptr(), device.stream()))
    q = device.empty(n)
    _lib.check(lib.pbh_fill_lhs(seed, n, 0, n, col, 1, q.data_ptr(), n, device.stream()))
    return out, torch.sort(q).values


def _cfg3_columns():
    from oracle.pipeline import cfg_dists

    return list(enumerate(cfg_dists(32)))


@pytest.mark.timeout(900)
def test_cfg3_values_1e8_sampled_vs_scipy(gpu):
    import torch

    from oracle.pipeline import ppf_columns
    from probabilit_amd import qmc

    seed = qmc.seed_from(0)  # the bench's first seed, as Node.sample hands it to the generators
    rng = np.random.default_rng(11)
    worst = {}
    for j, (name, kw) in _cfg3_columns():
        x, q = _sorted_columns(seed, N8, j, name, kw)
        t = torch.from_numpy(np.sort(rng.choice(N8, 1_000_000, replace=False))).to(x.device)
        xs, qs = x[t].cpu().numpy(), q[t].cpu().numpy()
        del x, q
        exp = ppf_columns(qs[:, None], [(name, kw)], threads=THREADS)[:, 0]
        if name == "poisson":
            np.testing.assert_array_equal(xs, exp, err_msg=f"column {j}")
        else:
            assert_close(xs, exp, rtol=RTOL, what=f"column {j} {name}{kw}")
            worst[j] = float(np.max(np.abs(xs - exp) / np.maximum(np.abs(exp), 1e-300)))
    print("max relative difference per continuous column:", worst)


@pytest.mark.timeout(900)
def test_cfg3_poisson_boundaries_1e8_every_stratum(gpu):
    import scipy.special as sc
    import torch

    from oracle.ppf import ppf as ref_ppf
    from probabilit_amd import qmc

    seed = qmc.seed_from(0)
    report = []
    for j, (name, kw) in _cfg3_columns():
        if name != "poisson":
            continue
        mu = kw["mu"]
        x, q = _sorted_columns(seed, N8, j, name, kw)
        k = np.arange(0, int(mu + 40 * np.sqrt(mu) + 40), dtype=np.float64)
        b = sc.pdtr(k, mu)
        b = b[(b > 0) & (b < 1)]
        lo = torch.searchsorted(q, torch.from_numpy(b * (1 - 1e-6)).to(q.device))
        hi = torch.searchsorted(q, torch.from_numpy(b * (1 + 1e-6)).to(q.device))
        idx = torch.cat([torch.arange(int(a), int(e), device=q.device) for a, e in zip(lo.tolist(), hi.tolist())])
        xs, qs = x[idx].cpu().numpy(), q[idx].cpu().numpy()
        del x, q
        exp = ref_ppf("poisson", qs, mu=mu)
        table = sc.pdtr(np.arange(0, int(mu + 60 * np.sqrt(mu) + 80), dtype=np.float64), mu)
        definition = np.searchsorted(table, qs, side="left").astype(np.float64)
        diff = xs != exp
        report.append({"column": j, "mu": mu, "strata_near_boundaries": int(idx.numel()),
                       "device_differs_from_scipy": int(diff.sum()),
                       "scipy_differs_from_definition": int(np.count_nonzero(exp != definition))})
    record("cfg3_poisson_boundaries_1e8", report)
    assert all(r["device_differs_from_scipy"] == 0 for r in report), report


@pytest.mark.timeout(600)
def test_cfg2_1e7_uncorrelated_vs_oracle(gpu):
    from oracle.pipeline import cfg_dists, ppf_columns
    from probabilit_amd import device, native, qmc
    from probabilit_amd.modeling import Distribution, NoOp

    n, d, seed = 10_000_000, 8, 0
    ds = [Distribution(nm, **kw) for nm, kw in cfg_dists(d)]
    NoOp(*ds).sample_device(n, random_state=seed, method="lhs")
    Q = native.fill_lhs(qmc.seed_from(seed), n, d)  # the native quantile matrix of this seed (row order)
    X = ppf_columns(Q, cfg_dists(d), threads=THREADS)
    del Q
    counts = {}
    for j, x in enumerate(ds):
        got = device.to_host(x.samples_device)
        if cfg_dists(d)[j][0] == "poisson":
            counts[j] = int(np.count_nonzero(got != X[:, j]))
        else:
            assert_close(got, X[:, j], rtol=RTOL, what=f"cfg2 column {j}")
    record("cfg2_1e7_poisson_vs_scipy", {"device_differs_from_scipy_per_poisson_column": counts})
    assert not any(counts.values()), counts


@pytest.mark.timeout(600)
def test_cfg5_1e8_fused_equals_per_node_and_oracle_block(gpu, monkeypatch):
    import torch

    from oracle.pipeline import mutual_fund
    from oracle.streams import sobol_closed_form
    from probabilit_amd import dag, qmc
    from probabilit_amd.modeling import Distribution

    n, years, seed = N8, 20, 3

    def fund():
        r = 0
        for _ in range(years):
            r = r * Distribution("norm", loc=1.11, scale=0.15) + 1200
        return r

    sinks = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("PBH_DAG", flag)
        before = dag.counts["fused"]
        s = fund().sample_device(n, random_state=seed, method="sobol", gc_strategy=[])
        assert (dag.counts["fused"] > before) == (flag == "1")
        sinks[flag] = s.clone()
        del s
    assert torch.equal(sinks["1"], sinks["0"])
    row0, m = 50_000_000, 1_000_000
    sv, shift = qmc.sobol_setup(years, seed, 30)
    Q = sobol_closed_form(np.asarray(sv), np.asarray(shift), m, bits=30, index0=row0)
    exp = mutual_fund(Q, years=years)
    assert_close(sinks["1"][row0:row0 + m].cpu().numpy(), exp, rtol=1e-13, what="cfg5 block vs oracle")
