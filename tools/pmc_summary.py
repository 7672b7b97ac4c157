"""Per-kernel HBM traffic from two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR > summary.json

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE reports half the
bytes of wide (16 B/lane) coalesced streaming reads (MI355X_MICROARCH.md, HBM section), so
`hbm_bytes` uses 2 x FETCH_SIZE + WRITE_SIZE; the raw values are kept alongside.
"""

import csv
import glob
import json
import os
import re
import sys


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != counter:
                continue
            name = row["Kernel_Name"]
            m = re.search(r"(k_\w+)(<[^>(]*>)?", name)
            key = (m.group(1) + (m.group(2) or "")) if m else name
            ent = per.setdefault(key, {})
            ent.setdefault(row["Dispatch_Id"], 0.0)
            ent[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in per.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out[k] = {"dispatches": max(nf, nw), "fetch_kib_raw": round(f, 1), "write_kib": round(w, 1),
                  "hbm_bytes": round((2 * f + w) * 1024)}
    json.dump({"unit": "bytes per dispatch", "correction": "hbm_bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950)",
               "kernels": out}, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
