set -o pipefail
# Round 4: microbenchmark, ppf/ic GPU tests, 10-step bench with the ppf sweep, then the interleaved
# A/B of the three step-3 / histogram switches.  TAG as $1.
TAG=${1:-r4c}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 tools/gpu/mbfeistel > gpurun_out/mbfeistel_$TAG.json 2>&1; echo "mbfeistel exit $?"; cat gpurun_out/mbfeistel_$TAG.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_ppf.py tests/test_gpu_ic.py tests/test_gpu_scale.py tests/test_gpu_dists.py tests/test_gpu_step4_gen.py -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json | head -24
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_APPLY_W2=1" "PBH_APPLY_NT=1" "PBH_HIST_BLOCKS=32" "PBH_HIST_BLOCKS=128"
