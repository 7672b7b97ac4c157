set -o pipefail
# ppf sweep A/B: block-wide tail queue (default) against the per-wave stacks (wq)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5zg
for r in 1 2; do
  for v in "" wq; do
    name=${v:-default}
    timeout -k 10 200 python -u tools/ppf_sweep.py ${v:+--variant $v} > gpurun_out/r5zg/sweep_${name}_$r.json 2> gpurun_out/r5zg/sweep_${name}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5zg/sweep_${name}_$r.json')); pd=d['per_dist']
print('$name', $r, round(d['frac'],4), {k[:26]: v['ms'] for k,v in pd.items() if 'norm' in k})"
  done
done
