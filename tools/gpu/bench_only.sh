set -o pipefail
# One bench line (10 steps) and its summary.  TAG as $1.
TAG=${1:-b}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_show.txt; head -22 gpurun_out/${TAG}_show.txt
