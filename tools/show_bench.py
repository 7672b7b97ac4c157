"""Print the headline, the ppf sweep and the per-kernel tables of a bench.py JSON line
(python tools/show_bench.py FILE)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value", d["value"], "Msamples/s  ms/step", d["ms_per_step"], " roofline", d["roofline"]["kernel"],
      d["roofline"]["frac"], " pipeline", (d.get("pipeline_roofline") or {}).get("frac"))
sw = d.get("ppf_sweep")
if sw:
    print("ppf sweep", sw["achieved"], "GB/s  frac", sw["frac"])
    for k, v in sw["per_dist"].items():
        print(f"   {k:44s} {v['ms']:.4f} ms {v['GBps']:8.1f} GB/s  {v['kernel']}")
for key in ("kernels_standalone", "kernels"):
    if key in d:
        print("--", key)
        for k, v in sorted(d[key].items(), key=lambda kv: -kv[1]["total_ms_per_step"]):
            print(f"{k:24s} {v['total_ms_per_step']:8.3f} ms/step {v['launches']:6d} launches  avg {v['avg_ms']:.4f} ms  "
                  f"{v['GBps']} GB/s")
