set -o pipefail
# Round-3 GPU step: the given tests (all reported, no -x), then a short bench and its kernel table.
# Usage: bash tools/gpu/r3.sh TAG "pytest args" [bench]
TAG=${1:-r3}; ARGS=$2; BENCH=$3
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest $ARGS -v -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}_tests.log | tail -60; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  echo "bench exit $?"; python3 tools/show_bench.py gpurun_out/${TAG}_bench.json | head -40
fi
