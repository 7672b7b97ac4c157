import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu on the GPU box")


def record(name, obj):
    """Print an at-scale measurement and keep it as JSON under gpurun_out/records/ (merged back
    from the GPU box; the committed copies live under profiles/)."""
    import json

    text = json.dumps(obj, indent=1, default=float)
    print(f"[record {name}] {text}")
    d = os.environ.get("PBH_RECORD_DIR", os.path.join(ROOT, "gpurun_out", "records"))
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"{name}.json"), "w") as f:
        f.write(text + "\n")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def assert_close(actual, expected, rtol=1e-10, atol=0.0, what=""):
    """Elementwise |a - e| <= atol + rtol * |e|, NaN == NaN and inf == inf of the same sign."""
    a = np.asarray(actual, dtype=float)
    e = np.asarray(expected, dtype=float)
    assert a.shape == e.shape, f"{what}: shape {a.shape} != {e.shape}"
    same_nan = np.isnan(a) & np.isnan(e)
    same_inf = np.isinf(a) & np.isinf(e) & (np.sign(a) == np.sign(e))
    with np.errstate(invalid="ignore"):
        ok = same_nan | same_inf | (np.abs(a - e) <= atol + rtol * np.abs(e))
    if not ok.all():
        bad = np.flatnonzero(~ok.ravel())[:8]
        raise AssertionError(f"{what}: {(~ok).sum()} of {ok.size} elements differ beyond rtol={rtol}; "
                             f"first at {bad}: actual={a.ravel()[bad]} expected={e.ravel()[bad]}")


@pytest.fixture(scope="session")
def gpu():
    import probabilit_amd.device as dev

    return dev.device()
