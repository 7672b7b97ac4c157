set -o pipefail
TAG=${1:-r4r}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ic.py tests/test_gpu_step4_gen.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider -k "not variants" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
bash tools/gpu/bench_only.sh $TAG
