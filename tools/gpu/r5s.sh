set -o pipefail
# Round 5: the reference stream's permutations on the stable radix sort: tests, timing, profile.
TAG=${1:-r5s}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py tests/test_gpu_ppf.py -m gpu -x -q -s -k "reference or cancellation" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; grep -E "passed|failed|ambiguous" gpurun_out/$TAG/tests.log | tail -4; [ $st -eq 0 ] || { grep -E "Error|FAIL|Mismatch" gpurun_out/$TAG/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/ref_lhs_time.py 10000000 32 3 > gpurun_out/$TAG/time_1e7.json 2>&1; echo "t $?"; tail -1 gpurun_out/$TAG/time_1e7.json
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o ref --output-format csv -- python3 tools/ref_stream_profile.py 2 > gpurun_out/$TAG/run.log 2>&1
echo "prof exit $?"; grep "call" gpurun_out/$TAG/run.log
