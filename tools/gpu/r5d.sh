set -o pipefail
# Round 5: windowed gamma sweep (k_ppf_gamma_w + slow list): ppf / dists / modeling GPU tests, bench.
TAG=${1:-r5d}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ppf.py tests/test_gpu_dists.py tests/test_gpu_modeling.py tests/test_gpu_streams.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.txt; head -14 gpurun_out/${TAG}_bench.txt
