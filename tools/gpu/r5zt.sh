set -o pipefail
# Round 5 at HEAD (strata-ordered reference-stream IC, materialised step 4 on lanes): the whole
# -m gpu suite, then the bench.
TAG=${1:-r5zt}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -2 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|FAIL" gpurun_out/$TAG/tests.log | head -20; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['reference_stream']['value'], d['reference_stream']['stream_only'], d['roofline']['frac'], d['ppf_sweep']['frac'])"
