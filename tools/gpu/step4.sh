set -o pipefail
# Step-4 iteration: the step-4 / IC / modeling GPU tests, then the bench.
TAG=${1:-s4}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ic.py tests/test_gpu_modeling.py tests/test_gpu_step4_buckets.py ${EXTRA_TESTS} -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
tail -12 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
stop_if_crashed $? bench
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json
