"""Bit-for-bit check of a library variant against the default on the kernels it changes: norm /
lognorm / poisson / gamma sweeps (pbh_ppf) and fused native-LHS columns (Node.sample, method="lhs").

    python tools/ab_bitexact.py VARIANT     # prints the number of differing elements per case
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys
import numpy as np
sys.path.insert(0, {root!r})
from probabilit_amd import _lib
if {variant!r} != "default":
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libprobabilit_hip_{variant}.so")
from probabilit_amd import native
from probabilit_amd.modeling import Distribution as D
q = np.concatenate([np.random.default_rng(5).random(3_000_000), [1e-300, 1e-20, 0.5, 1 - 1e-16, 0.0, 1.0]])
out = {{}}
for name, kw in [("norm", dict(loc=0.0, scale=1.0)), ("norm", dict(loc=5.0, scale=2.0)), ("lognorm", dict(s=0.5)),
                 ("lognorm", dict(s=2.0, loc=-1.0, scale=3.0)), ("poisson", dict(mu=4.0)), ("poisson", dict(mu=30.0)),
                 ("poisson", dict(mu=250.0, loc=2.0)), ("gamma", dict(a=2.0))]:
    out[f"ppf_{{name}}_{{sorted(kw.items())}}"] = native.ppf(name, q, **kw)
    out[f"lhs_{{name}}_{{sorted(kw.items())}}"] = D(name, **kw).sample(2_000_003, method="lhs", random_state=9)
np.savez({path!r}, **out)
"""


def run(variant, path):
    p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, variant=variant, path=path)],
                       capture_output=True, text=True, timeout=600)
    if p.returncode:
        print(p.stderr[-2000:])
        sys.exit(p.returncode)


v = sys.argv[1]
run("default", "/tmp/ab_default.npz")
run(v, "/tmp/ab_variant.npz")
a, b = np.load("/tmp/ab_default.npz"), np.load("/tmp/ab_variant.npz")
bad = 0
for k in a.files:
    d = int((~((a[k] == b[k]) | (np.isnan(a[k]) & np.isnan(b[k])))).sum())
    bad += d
    print(k, "differing:", d)
print("TOTAL differing:", bad)
sys.exit(1 if bad else 0)
