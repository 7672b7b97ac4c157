set -o pipefail
# Interleaved A/B of environment knobs, two rounds: bash tools/gpu/ab_env.sh TAG "ENV0" "ENV1" ...
# ("-" = defaults).  5-step bench per run, no CPU baseline / e2e / ppf sweep.
TAG=$1; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for E in "$@"; do
    [ "$E" = "-" ] && E="PBH_AB_DEFAULT=1"
    env $E timeout -k 10 300 python bench.py --no-cpu --no-e2e --ppf-rows 0 --steps 5 > gpurun_out/${TAG}_${i}_$rep.json 2> gpurun_out/${TAG}_${i}_$rep.err || exit 1
    python3 - gpurun_out/${TAG}_${i}_$rep.json "$E" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); ks = d["kernels_standalone"]
print(sys.argv[2], "ms", d["ms_per_step"], " ".join(f"{k}={v['total_ms_per_step']:.2f}" for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["total_ms_per_step"])[:8]))
PY
    i=$((i+1))
  done
done
