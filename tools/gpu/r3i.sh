set -o pipefail
# GPU tests + interleaved A/B of step-4 kernel variants.  Usage: bash tools/gpu/r3i.sh TAG "ENV_A" "ENV_B" ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_${i}_${rep}.json 2> gpurun_out/${TAG}_${i}_${rep}.err || exit $?
    python3 - "$rep" "$cfg" "gpurun_out/${TAG}_${i}_${rep}.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[3]))
ks = d["kernels_standalone"]
print(sys.argv[1], "[%s]" % sys.argv[2], d["ms_per_step"], " ".join("%s=%.2f" % (k, v["total_ms_per_step"]) for k, v in sorted(ks.items(), key=lambda kv: -kv[1]["total_ms_per_step"])))
PY
  done
done
