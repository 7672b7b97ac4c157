set -o pipefail
# Round 4: microbenchmark, key GPU tests, 5-step bench with the ppf sweep.  TAG as $1.
TAG=${1:-r4b}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 tools/gpu/mbfeistel > gpurun_out/mbfeistel_$TAG.json 2>&1; echo "mbfeistel exit $?"; cat gpurun_out/mbfeistel_$TAG.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_ppf.py tests/test_gpu_ic.py tests/test_gpu_step4_gen.py tests/test_gpu_scale.py tests/test_gpu_dists.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json | head -30
