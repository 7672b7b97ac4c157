set -o pipefail
# Round 5: k_finish_q pass-1 walk over the lane's bins together: step-4 tests, bench (standalone k_finish).
TAG=${1:-r5n}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_step4_buckets.py tests/test_gpu_ic.py tests/test_gpu_certificate.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -2 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/$TAG/tests.log | head -30; exit 1; }
for i in 1 2; do
timeout -k 10 400 python -u bench.py --no-e2e > gpurun_out/$TAG/bench$i.json 2> gpurun_out/$TAG/bench$i.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench$i.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels_standalone'].items()})"
done
