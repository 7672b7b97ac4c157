set -o pipefail
# Round 5: the reference LHS stream's device decode: tests, timing, kernel-trace profile at 1e7 x 32.
TAG=${1:-r5h}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_streams.py -m gpu -x -v -s -k "reference" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; grep -E "FAIL|ambiguous|rror" gpurun_out/$TAG/tests.log | head -40; [ $st -eq 0 ] || { tail -40 gpurun_out/$TAG/tests.log; exit 1; }
timeout -k 10 300 python -u tools/ref_lhs_time.py 10000000 32 3 > gpurun_out/$TAG/time_1e7.json 2>&1; echo "t2 $?"; tail -4 gpurun_out/$TAG/time_1e7.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o ref --output-format csv -- python3 tools/ref_lhs_time.py 10000000 32 2 > gpurun_out/$TAG/prof.log 2>&1
echo "prof exit $?"
f=$(find gpurun_out/$TAG/prof -name "*kernel_stats.csv" | head -1); echo $f; cut -d, -f1-8 "$f" | head -30
