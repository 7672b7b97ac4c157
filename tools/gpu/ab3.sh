set -o pipefail
# A/B of bench configurations given as env assignments, interleaved twice.
# Usage: bash tools/gpu/ab3.sh TAG "ENV_A" "ENV_B" ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
for rep in 1 2; do
  i=0
  for cfg in "$@"; do
    i=$((i+1))
    env $cfg timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_${i}_${rep}.json 2> gpurun_out/${TAG}_${i}_${rep}.err || exit $?
    echo "$rep [$cfg] $(python3 -c "import json;d=json.load(open('gpurun_out/${TAG}_${i}_${rep}.json'));print(d['ms_per_step'])")"
  done
done
