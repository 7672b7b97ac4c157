"""Interleaved A/B of bench.py's cfg3 step (N = 1e8, d = 32, LHS + ppf + Iman-Conover) across library
variants built by `python -m probabilit_amd.build --variant NAME -D ...` (--refstream: bench.py's
reference_stream workload, the same graph at 1e7 rows on stream="reference"): each variant runs in
its own process (the library loads once), alternating, and prints its ms per step.
python tools/ab_step.py [--rounds 2] [--steps 4] default sg128 ..."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import os, sys, time, json
sys.path.insert(0, {root!r})
from probabilit_amd import _lib
if {variant!r} != "default":
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), "libprobabilit_hip_{variant}.so")
import torch
import numpy as np
import probabilit_amd  # noqa: F401
from probabilit_amd import device
from probabilit_amd.modeling import Distribution, NoOp
dev = device.device()
base = [("norm", {{"loc": 0.0, "scale": 1.0}}), ("gamma", {{"a": 2.0}}), ("triang", {{"c": 0.3}}),
        ("poisson", {{"mu": 4.0}}), ("norm", {{"loc": 5.0, "scale": 2.0}}), ("gamma", {{"a": 0.7, "scale": 3.0}}),
        ("triang", {{"c": 0.8, "loc": 1.0, "scale": 2.0}}), ("poisson", {{"mu": 30.0}})]
dists = (base * 4)[:32]
A = np.random.default_rng(0).normal(size=(64, 32))
C = 0.9 * np.corrcoef(A, rowvar=False) + 0.1 * np.eye(32)
ds = [Distribution(name, **kw) for name, kw in dists]
if {op!r}:  # bench.py's operator_ic: ImanConover().set_target(C)(X) on a device-resident (1e8, 32) X
    from probabilit_amd.correlation import ImanConover
    NoOp(*ds).sample_device(100_000_000, random_state=3, method="lhs")
    X = torch.stack([x.samples_device for x in ds], dim=1)
    for x in ds:
        del x.samples_
    inst = ImanConover().set_target(C)
    run = lambda i: inst(X)
else:
    root = NoOp(*ds).correlate(*ds, corr_mat=C)
    kw = dict(method="lhs", stream="reference") if {ref!r} else dict(method="lhs")
    rows = 10_000_000 if {ref!r} else 100_000_000
    run = lambda i: root.sample_device(rows, random_state=i, **kw)
out = run(0)
del out
torch.cuda.synchronize(dev)
t = time.perf_counter()
for i in range({steps}):
    out = run(1 + i)
    del out
torch.cuda.synchronize(dev)
print(json.dumps({{"variant": {variant!r}, "ms": round(1e3 * (time.perf_counter() - t) / {steps}, 2)}}), flush=True)
"""

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--refstream", action="store_true", help="the reference-stream side figure (1e7 rows) instead")
ap.add_argument("--operator", action="store_true", help="bench.py's operator_ic (ImanConover()(X), 1e8 x 32) instead")
ap.add_argument("variants", nargs="+")
a = ap.parse_args()
out = []
for r in range(a.rounds):
    for v in a.variants:
        lib, *envs = v.split("+")  # "NAME+VAR=VALUE+...": library variant NAME with those env settings
        env = dict(os.environ, **dict(e.split("=", 1) for e in envs))
        p = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT, variant=lib, steps=a.steps, ref=a.refstream, op=a.operator)],
                           capture_output=True, text=True, timeout=600, env=env)
        if p.returncode != 0:
            print(p.stderr[-2000:], file=sys.stderr)
            sys.exit(p.returncode)
        out.append(dict(json.loads(p.stdout.strip().splitlines()[-1]), variant=v))
        print(json.dumps(out[-1]), flush=True)
print(json.dumps({"runs": out}))
