"""Print the headline and per-kernel table of a bench.py JSON line (python tools/show_bench.py FILE)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value", d["value"], "Msamples/s  ms/step", d["ms_per_step"], " roofline", d["roofline"]["kernel"],
      d["roofline"]["frac"], " pipeline", (d.get("pipeline_roofline") or {}).get("frac"))
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["total_ms_per_step"]):
    print(f"{k:24s} {v['total_ms_per_step']:8.3f} ms/step {v['launches']:6d} launches  avg {v['avg_ms']:.4f} ms  {v['GBps']} GB/s")
