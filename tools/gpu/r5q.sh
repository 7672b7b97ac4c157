set -o pipefail
# Round 5: invgamma / t on gamma's and beta's guides: dist tests, ext sweep.
TAG=${1:-r5q}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_dists.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -2 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|FAIL|mismatch|Max" gpurun_out/$TAG/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/ext_sweep.py > gpurun_out/$TAG/ext_sweep.json 2>&1; echo "ext exit $?"; tail -1 gpurun_out/$TAG/ext_sweep.json
