set -o pipefail
# extended sweep A/B: gamma-family fallbacks inline (default) against behind a call (cold)
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5zh
for r in 1 2; do
  for v in default cold; do
    timeout -k 10 300 python -u tools/ext_sweep.py 10000000 $([ $v = cold ] && echo cold) > gpurun_out/r5zh/ext_${v}_$r.json 2> gpurun_out/r5zh/ext_${v}_$r.err || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5zh/ext_${v}_$r.json').read().strip().splitlines()[-1]); s=d['sweep_ms']
print('$v', $r, {k[:18]: v for k,v in s.items() if any(x in k for x in ('chi','maxwell','nakagami','invgamma'))})"
  done
done
