set -o pipefail
# Round 4: every GPU test at HEAD, one process, each test under a thread timeout; log kept.
# Usage: bash tools/gpu/r4tests.sh TAG [pytest selection...]
TAG=${1:-r4tests}; shift
SEL=${@:-tests}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest $SEL -m gpu -v -rf --durations 25 --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -40 gpurun_out/${TAG}.log; exit $rc
