set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/r3e.sh r3e || exit $?
timeout -k 10 1100 python -u -m pytest tests/test_gpu_scale_values.py tests/test_gpu_scale.py -v -s -rf --timeout 1200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3f_scale.log 2>&1
rc=$?; echo "scale pytest exit $rc"; grep -E "PASSED|FAILED|ERROR|poisson|max relative|violations|mismatch" gpurun_out/r3f_scale.log | tail -20
