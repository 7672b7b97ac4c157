set -o pipefail
# Round 6: the default bench line at HEAD (what the driver runs), written under gpurun_out/<tag>/.
TAG=${1:-r6a}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u bench.py "${@:2}" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; st=$?
echo "bench exit $st"; [ $st -eq 0 ] || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
python3 tools/show_bench.py gpurun_out/$TAG/bench.json || true
