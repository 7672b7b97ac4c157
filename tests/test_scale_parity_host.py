"""The N=1e8 step-4 gate's classification (tests/scale_parity.py column_gate) on hand-made
columns: adjacent-rank swaps, device ties, reference ties, and real violations."""

import numpy as np

import scale_parity as sp


def _case():
    cs = np.array([0.1, 0.5, 0.3, 0.7, 0.9, 0.7, 0.2, 0.4, 0.6, 0.8])
    sx = np.arange(10, dtype=float) * 10
    return cs, sx, sx[sp._rank_minus_one(cs)].copy()


def test_exact_match():
    cs, sx, y = _case()
    assert sp.column_gate(0, cs, y, sx)["mismatched_rows"] == 0


def test_reference_tie_group():
    """Rows 3 and 5 tie exactly in the reference (both get int(7.5) - 1 = 6); a device whose CS
    differ by an ulp gives them positions 6 and 7."""
    cs, sx, y = _case()
    y[5] = 70.0
    out = sp.column_gate(0, cs, y, sx)
    assert out["violations"] == 0 and out["ties"] == 1 and out["pairs"][0]["kind"] == "ref_tie"


def test_swap_and_device_tie():
    cs = np.array([0.1, 0.2, 0.2 + 2 ** -55, 0.9])  # rows 1, 2 an ulp apart in the reference
    sx = np.array([1.0, 2.0, 3.0, 4.0])
    y = np.array([1.0, 3.0, 2.0, 4.0])  # swapped
    out = sp.column_gate(0, cs, y, sx)
    assert out["violations"] == 0 and out["swaps"] == 1
    y = np.array([1.0, 2.0, 2.0, 4.0])  # the device tied them: both get position 1
    out = sp.column_gate(0, cs, y, sx)
    assert out["violations"] == 0 and out["ties"] == 1


def test_violation():
    cs = np.array([0.1, 0.2, 0.5, 0.9])
    sx = np.array([1.0, 2.0, 3.0, 4.0])
    y = np.array([1.0, 3.0, 2.0, 4.0])  # rows 1, 2 are far apart in CS: a wrong rank
    assert sp.column_gate(0, cs, y, sx)["violations"] == 2
