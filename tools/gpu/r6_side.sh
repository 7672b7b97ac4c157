set -o pipefail
# Round 6: the operator / reference-stream side workloads at N rows under rocprofv3 (one stream),
# summaries under gpurun_out/<tag>/: bash tools/gpu/r6_side.sh TAG ROWS
TAG=${1:-r6s}; ROWS=${2:-100000000}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for w in operator refstream; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$w -o run --output-format csv -- python3 tools/side_profile.py $w $ROWS 2 > gpurun_out/$TAG/side_$w.log 2>&1 || { echo "$w failed"; tail -20 gpurun_out/$TAG/side_$w.log; exit 1; }
  grep "call" gpurun_out/$TAG/side_$w.log
done
find gpurun_out/$TAG -name "*kernel_stats.csv" | head
