"""Timeline of the last bench step from a rocprofv3 kernel trace (tools/gpu/timeline.sh):
per stream and kernel family, the first start, last end and summed busy time relative to the
step's first kernel, plus gaps on the caller's stream.  python tools/timeline.py TRACE.csv [steps]"""
import csv
import re
import sys
from collections import defaultdict

FAMILIES = [("tables", r"k_gamma_guide|k_poisson_(table|guide)"), ("counts", r"k_lhs_sorted_ppf"),
            ("heads", r"k_sort_heads"), ("scores", r"k_perm_scores"), ("means", r"k_means|k_colsum"),
            ("gram", r"k_gram"), ("apply", r"k_apply|k_transform_matrix"), ("hist16", r"k_hist16"),
            ("adapt", r"k_adapt_reset|k_seg_hist|k_seg_map|k_make_codes_adapt"), ("codes", r"k_make_codes"),
            ("msd1", r"k_msd1"), ("msd2", r"k_msd2"), ("finish", r"k_finish"), ("place_msd", r"k_place_msd"),
            ("place_gen", r"k_place_gen|k_place_positions"), ("general", r"k_onesweep|k_scatter|k_place\b|k_code|k_runs"),
            ("rccl", r"nccl|rccl|ncclDevKernel"), ("copy", r"copyBuffer|fillBuffer")]


def family(name):
    for f, rx in FAMILIES:
        if re.search(rx, name):
            return f
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
gam = [i for i, r in enumerate(rows) if "k_gamma_guide" in r["Kernel_Name"]]
per = len(gam) // steps
first = gam[-per] if per else 0
step = rows[first:]
t0 = int(step[0]["Start_Timestamp"])
tab = defaultdict(lambda: [1e30, 0, 0.0, 0])
for r in step:
    a, b = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    k = (r["Stream_Id"], family(r["Kernel_Name"]))
    e = tab[k]
    e[0], e[1], e[2], e[3] = min(e[0], a), max(e[1], b), e[2] + (b - a), e[3] + 1
end = max(v[1] for v in tab.values())
print(f"last step: {end / 1e6:.2f} ms, {len(step)} kernels")
for (st, f), (a, b, busy, cnt) in sorted(tab.items(), key=lambda kv: kv[1][0]):
    print(f"stream {st:>3s} {f:10s} {a / 1e6:8.2f} .. {b / 1e6:8.2f} ms  busy {busy / 1e6:7.2f} ms  {cnt:5d} kernels")

# device idle time inside the step: the gaps in the union of every kernel's [start, end), with the
# kernels on either side of the largest ones (host synchronisations, launch latency)
iv = sorted((int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0, r["Kernel_Name"]) for r in step)
gaps, cur_end, prev = [], iv[0][1], iv[0][2]
for a, b, nm in iv[1:]:
    if a > cur_end:
        gaps.append((a - cur_end, cur_end, prev[:40], nm[:40]))
    if b > cur_end:
        cur_end, prev = b, nm
idle = sum(g[0] for g in gaps)
print(f"device idle inside the step: {idle / 1e6:.2f} ms in {len(gaps)} gaps (busy union {(end - idle) / 1e6:.2f} ms)")
for g, at, before, after in sorted(gaps, reverse=True)[:12]:
    print(f"  gap {g / 1e3:8.1f} us at {at / 1e6:8.2f} ms  after {before}  before {after}")
prev_steps = rows[:first]
if prev_steps:
    last_prev = max(int(r["End_Timestamp"]) for r in prev_steps)
    print(f"gap from the previous step's last kernel: {(t0 - last_prev) / 1e3:.1f} us")
