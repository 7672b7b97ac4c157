set -o pipefail
# One build-measure iteration on the GPU box: GPU tests, bench, rocprofv3 kernel stats.
# Ordinary failures (exit 1) continue; a crash, abort or time limit ends the script.
TAG=${1:-rX}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
stop_if_crashed $? bench
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
stop_if_crashed $? prof
if [ -n "$PMC" ]; then bash $R/tools/gpu/pmc.sh $TAG; fi
