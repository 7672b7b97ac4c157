set -o pipefail
# Evidence run (tools/gpu/r3final.sh) followed by interleaved A/B bench runs of the given
# configurations (bench.py --steps 5 --warmup 2, standalone kernel times per run).
# Usage: bash tools/gpu/r3ab_final.sh TAG "ENV_A" "ENV_B" ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/r3final.sh $TAG || exit $?
cd $R
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_ab_${i}_${rep}.json 2> gpurun_out/${TAG}_ab_${i}_${rep}.err || exit $?
    python3 - "$rep" "$cfg" "gpurun_out/${TAG}_ab_${i}_${rep}.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
ks = d["kernels_standalone"]
print(sys.argv[1], "[%s]" % sys.argv[2], d["ms_per_step"], " ".join("%s=%.2f" % (k, v["total_ms_per_step"]) for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["total_ms_per_step"])))
PY
  done
done
