"""Per-kernel issue-level summary of the rocprofv3 passes of tools/gpu/pmc_valu.sh.

    python tools/pmc_valu_summary.py OUTDIR > summary.json

For every kernel (name up to its template arguments) and every counter: the mean per dispatch
(summed over the counter's instances).  Derived, per dispatch:

* duration_ms: the kernel-trace mean (the counters' own run);
* cycles = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md);
* valu_busy = 4 SQ_ACTIVE_INST_VALU / (1024 SIMDs x cycles): the fraction of SIMD cycles that
  issued a vector instruction (SQ_ACTIVE_INST_* count quad-cycles; the gfx94x VALUBusy
  formula with the gfx950 GRBM correction);
* wave_active = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, wave_wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES,
  wave_issue_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES;
* f64_gflops: 64 lanes x (2 FMA + MUL + ADD + TRANS f64 instructions) / duration, against the
  78.6 TFLOP/s FP64 vector peak (f64_frac).
"""

import csv
import glob
import json
import os
import re
import sys

SIMDS = 1024
F64_PEAK_GFLOPS = 78600.0


def key_of(name):
    m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name


def load_counters(d):
    per = {}  # kernel -> counter -> dispatch -> value
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = key_of(row["Kernel_Name"])
            c = row["Counter_Name"]
            per.setdefault(k, {}).setdefault(c, {}).setdefault(row["Dispatch_Id"], 0.0)
            per[k][c][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in per.items()}, \
        {k: max(len(v) for v in cs.values()) for k, cs in per.items()}


def load_durations(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = key_of(row["Kernel_Name"])
            per.setdefault(k, []).append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    root = sys.argv[1]
    out = {}
    for run in sorted(os.listdir(root)):
        d = os.path.join(root, run)
        if not os.path.isdir(d):
            continue
        ctr, disp = load_counters(d)
        dur = load_durations(d)
        for k, cs in ctr.items():
            e = out.setdefault(run.rsplit("_p", 1)[0], {}).setdefault(k, {"dispatches": disp[k]})
            e.update({c: round(v, 1) for c, v in cs.items()})
            if k in dur:
                e["duration_ms"] = round(dur[k], 4)
    for run, ks in out.items():
        for k, e in ks.items():
            g = e.get("GRBM_GUI_ACTIVE")
            if g and "SQ_ACTIVE_INST_VALU" in e:
                e["valu_busy"] = round(4 * e["SQ_ACTIVE_INST_VALU"] / (SIMDS * g / 8), 4)
            wc = e.get("SQ_WAVE_CYCLES")
            if wc:
                for src, dst in (("SQ_ACTIVE_INST_ANY", "wave_active"), ("SQ_WAIT_ANY", "wave_wait"),
                                 ("SQ_WAIT_INST_ANY", "wave_issue_stall")):
                    if src in e:
                        e[dst] = round(e[src] / wc, 4)
            f64 = [e.get(c) for c in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                      "SQ_INSTS_VALU_TRANS_F64")]
            if all(v is not None for v in f64) and e.get("duration_ms"):
                flops = 64 * (2 * f64[0] + f64[1] + f64[2] + f64[3])
                e["f64_gflops"] = round(flops / (e["duration_ms"] / 1e3) / 1e9, 1)
                e["f64_frac"] = round(e["f64_gflops"] / F64_PEAK_GFLOPS, 4)
    json.dump({"what": "per-dispatch means of rocprofv3 PMC passes (tools/gpu/pmc_valu.sh); derived fields: "
                       "see tools/pmc_valu_summary.py", "runs": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
