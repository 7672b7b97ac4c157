set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_step4_gen.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3d_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r3d_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab3.sh ab3 "PBH_X=1" "GPU_MAX_HW_QUEUES=4" || exit $?
