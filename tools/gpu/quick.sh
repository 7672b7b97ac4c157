set -o pipefail
# Targeted GPU step: pytest on the given test paths / -k expression, then optionally the bench.
# Usage: bash tools/gpu/quick.sh TAG "pytest args" [bench]
TAG=${1:-rX}; ARGS=$2; BENCH=$3
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest $ARGS ${XFLAG--x} -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
  echo "bench exit $?"
fi
