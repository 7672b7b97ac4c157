set -o pipefail
# Round 5: reference stream on the device: streams + distributed tests, then a bench line.
TAG=${1:-r5j}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_distributed.py tests/test_gpu_modeling.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -3 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/$TAG/tests.log | head -30; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['reference_stream'], d['roofline']['frac'], d['ppf_sweep']['frac'])"
