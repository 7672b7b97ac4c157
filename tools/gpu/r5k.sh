set -o pipefail
TAG=${1:-r5k}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$TAG/prof -o cfg2 --output-format csv -- python3 tools/cfg2_trace.py 10 > gpurun_out/$TAG/run.log 2>&1
echo "exit $?"; grep wall gpurun_out/$TAG/run.log
