set -o pipefail
# A/B bench of environment knobs: bash tools/gpu/bench_ab.sh TAG "ENV1" "ENV2" ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
i=0
for E in "$@"; do
  env $E timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.err
  rc=$?; echo "ab$i [$E] exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  i=$((i+1))
done
