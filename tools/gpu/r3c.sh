set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_step4_gen.py tests/test_gpu_scale.py tests/test_gpu_ic.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r3c_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab3.sh ab2 "PBH_COUNTS_STREAM=0" "PBH_COUNTS_STREAM=0 GPU_MAX_HW_QUEUES=8" || exit $?
timeout -k 10 400 python tools/rank_budget.py > gpurun_out/r3c_budget.json 2> gpurun_out/r3c_budget.err; echo "budget exit $?"; cat gpurun_out/r3c_budget.json
