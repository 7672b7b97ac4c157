set -o pipefail
TAG=${1:-r5r}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppf.py -m gpu -x -q -k "cancellation" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1; st=$?; echo "pytest $st"; tail -2 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|Mismatch|Max" gpurun_out/$TAG/tests.log | head; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o ref --output-format csv -- python3 tools/ref_stream_profile.py 2 > gpurun_out/$TAG/run.log 2>&1
echo "prof exit $?"; grep "call" gpurun_out/$TAG/run.log
