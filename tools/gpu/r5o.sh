set -o pipefail
# Round 5: the full GPU suite at HEAD (-s: the at-scale tests print their records), then a bench line.
TAG=${1:-r5o}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q -s -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/gpu_tests.txt 2>&1
st=$?; echo "pytest exit $st"; tail -3 gpurun_out/$TAG/gpu_tests.txt; [ $st -eq 0 ] || { grep -E "Error|FAIL" gpurun_out/$TAG/gpu_tests.txt | head -20; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['reference_stream']['value'], d['roofline']['frac'], d['ppf_sweep']['frac'])"
