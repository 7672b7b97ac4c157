set -o pipefail
TAG=${1:-r4p}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
bash tools/gpu/r4p.sh $TAG || exit $?
timeout -k 10 300 python tools/profile_host.py 100000000 3 > gpurun_out/${TAG}_host.txt 2>&1
echo "host exit $?"; head -50 gpurun_out/${TAG}_host.txt
