set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_step4_gen.py tests/test_gpu_scale.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r3b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err
echo "bench exit $?"; python3 tools/show_bench.py gpurun_out/r3b_bench.json | head -14
bash tools/gpu/timeline.sh r3b
