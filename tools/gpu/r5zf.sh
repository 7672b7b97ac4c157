set -o pipefail
# ppf sweep A/B of the poisson kernel shape: default, 8 items per thread, 4096 blocks, 2 items x 4096 blocks
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5zf
for r in 1 2; do
  for v in "" p8 g4k p2g4k; do
    name=${v:-default}
    timeout -k 10 200 python -u tools/ppf_sweep.py ${v:+--variant $v} > gpurun_out/r5zf/sweep_${name}_$r.json 2> gpurun_out/r5zf/sweep_${name}_$r.err || exit 1
    python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5zf/sweep_${name}_$r.json')); pd=d['per_dist']
print('$name', $r, round(d['frac'],4), {k[:22]: v['ms'] for k,v in pd.items() if 'poisson' in k})"
  done
done
