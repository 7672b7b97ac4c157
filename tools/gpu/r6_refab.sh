set -o pipefail
# Round 6: the reference stream alone (tools/ref_lhs_time.py 1e7 x 32), library variants interleaved
TAG=${1:-r6ra}; shift
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
for r in 1 2 3; do for v in "$@"; do
  timeout -k 10 300 python3 tools/ref_lhs_time.py 10000000 32 3 $v > gpurun_out/$TAG/t_${v}_$r.json 2> gpurun_out/$TAG/t_${v}_$r.err || { tail -5 gpurun_out/$TAG/t_${v}_$r.err; exit 1; }
  echo "$v $(tail -1 gpurun_out/$TAG/t_${v}_$r.json | python3 -c 'import json,sys; d=json.load(sys.stdin); print([x["ms"] for x in d["runs"]])')"
done; done
