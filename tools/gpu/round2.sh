set -o pipefail
# Round-2 GPU step: full GPU suite (new at-scale parity tests included), the all-column N=1e8
# step-4 gate, then the bench.  Ordinary failures (exit 1) continue; a crash, abort or time
# limit ends the script.
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
tail -15 gpurun_out/${TAG}_tests.log
if [ -z "$SKIP_PARITY" ]; then
  timeout -k 10 600 python -u tools/parity_1e8.py --out gpurun_out/${TAG}_parity_1e8.json > gpurun_out/${TAG}_parity_1e8.log 2>&1
  stop_if_crashed $? parity
fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
stop_if_crashed $? bench
