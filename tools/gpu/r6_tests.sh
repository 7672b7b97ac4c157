set -o pipefail
# Round 6: a subset (or all) of the -m gpu tests: bash tools/gpu/r6_tests.sh TAG [pytest args...]
TAG=${1:-r6t}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
shift
timeout -k 10 1100 python -u -m pytest -m gpu -x -v -s -rf --timeout 600 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -3 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/$TAG/tests.log | head -30; exit 1; }
