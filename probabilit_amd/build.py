"""Build libprobabilit_hip.so (gfx950 only) in-tree with hipcc.

    python -m probabilit_amd.build            # incremental
    python -m probabilit_amd.build --force    # rebuild everything

Every csrc/*.hip translation unit is compiled to an object for --offload-arch=gfx950 with
-ffp-contract=off (each multiply/add rounds separately, as in scipy/numpy's x86-64 builds;
FMA only where a kernel asks for it explicitly) and linked into one shared library next to
this file.  The .so is git-ignored but travels to the GPU box with the repo snapshot.
"""

import argparse
import concurrent.futures
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(HERE, "..", "include")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libprobabilit_hip.so")
ARCH = "gfx950"

CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}",
            "-Wall", "-Wno-unused-function", "-Wno-unused-variable", "-I", CSRC, "-I", INCLUDE]


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the native library needs ROCm's hipcc (gfx950)")


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".inc"))]
    hs.append(os.path.join(INCLUDE, "probabilit_hip.h"))
    return hs


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False, variant=None, defines=()):
    """variant: build libprobabilit_hip_<variant>.so with extra -D `defines` (A/B measurements:
    a measuring tool points probabilit_amd._lib.LIB_PATH at it before the first load); the
    default library is untouched."""
    bdir = BUILD if not variant else BUILD + "_" + variant
    lib_path = LIB if not variant else os.path.join(HERE, f"libprobabilit_hip_{variant}.so")
    os.makedirs(bdir, exist_ok=True)
    cc = hipcc()
    headers = _headers()
    objs, jobs = [], []
    extra = [f"-D{d}" for d in defines]
    for src in _sources():
        obj = os.path.join(bdir, os.path.basename(src).replace(".hip", ".o"))
        objs.append(obj)
        if force or _stale(obj, [src] + headers):
            jobs.append([cc, *CXXFLAGS, *extra, "-c", src, "-o", obj])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {cmd[-3]}:\n{r.stdout}\n{r.stderr}")
        return r.stderr

    workers = min(8, max(1, len(jobs)))
    with concurrent.futures.ThreadPoolExecutor(workers) as ex:
        for warn in ex.map(run, jobs):
            if warn and verbose:
                print(warn, file=sys.stderr)
    if force or jobs or _stale(lib_path, objs):
        run([cc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", lib_path, *objs])
    return lib_path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--variant", default=None, help="build libprobabilit_hip_<variant>.so")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra preprocessor define")
    a = ap.parse_args()
    print(build(force=a.force, verbose=a.verbose, variant=a.variant, defines=a.defines))
