set -o pipefail
# Round 4: discrete columns placed from their run tables (k_place_gen_runs).  The new test, the
# generated-column / IC / distributed tests, then the A/B against per-row evaluation (PBH_PLACE_RUNS=0).
TAG=${1:-r4i}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py -k "runs" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_runs.log 2>&1
rc=$?; echo "runs pytest exit $rc"; tail -8 gpurun_out/${TAG}_runs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ic.py tests/test_gpu_dists.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_PLACE_RUNS=0" || exit $?
