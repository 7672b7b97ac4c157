set -o pipefail
# Round 6: the ppf sweep of each library variant, interleaved: bash tools/gpu/r6_ppfab.sh TAG VARIANT...
TAG=${1:-r6pa}; shift
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
for r in 1 2; do for v in "$@"; do
  a=""; [ "$v" = default ] || a="--variant $v"
  timeout -k 10 300 python3 tools/ppf_sweep.py $a > gpurun_out/$TAG/sweep_${v}_$r.json 2> gpurun_out/$TAG/sweep_${v}_$r.err || { tail -5 gpurun_out/$TAG/sweep_${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['frac'], {k[:22]: v['ms'] for k, v in d['per_dist'].items()})" gpurun_out/$TAG/sweep_${v}_$r.json $v
done; done
