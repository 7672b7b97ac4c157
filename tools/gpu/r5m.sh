set -o pipefail
TAG=${1:-r5m}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 200 python -u tools/cfg2_overhead.py 1000 200 > gpurun_out/$TAG/o1k.json 2>&1; echo "e $?"; tail -1 gpurun_out/$TAG/o1k.json
timeout -k 10 200 python -u tools/cfg2_overhead.py 10000000 30 > gpurun_out/$TAG/o1e7.json 2>&1; echo "e $?"; tail -1 gpurun_out/$TAG/o1e7.json
