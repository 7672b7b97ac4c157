set -o pipefail
# Round 5: the device decode of the reference LHS stream: tests, then timing at 1e6 x 32 and 1e7 x 32.
TAG=${1:-r5g}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -v -s -k "reference" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; grep -E "PASS|FAIL|ambiguous|Error|error" gpurun_out/$TAG/tests.log | head -40; [ $st -eq 0 ] || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
timeout -k 10 200 python -u tools/ref_lhs_time.py 1000000 32 2 > gpurun_out/$TAG/time_1e6.json 2>&1; echo "t1 $?"; cat gpurun_out/$TAG/time_1e6.json
timeout -k 10 300 python -u tools/ref_lhs_time.py 10000000 32 3 > gpurun_out/$TAG/time_1e7.json 2>&1; echo "t2 $?"; cat gpurun_out/$TAG/time_1e7.json
