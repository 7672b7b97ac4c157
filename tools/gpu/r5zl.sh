set -o pipefail
# cfg2 wall per call at 1e7 with 2 / 3 (default) / 4 side streams for the grouped leaves
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/r5zl
for r in 1 2; do
  for L in 3 4 2; do
    PBH_STEP4_STREAMS=$L timeout -k 10 200 python -u tools/profile_cfg2.py 40 > gpurun_out/r5zl/cfg2_L${L}_$r.txt 2>&1 || exit 1
    python3 -c "
import json; t=open('gpurun_out/r5zl/cfg2_L${L}_$r.txt').read(); i=t.index('{'); j=t.index('\n}\n', i)+2; d=json.loads(t[i:j])
print('lanes $L round $r', d['10000000']['wall_ms_untimed'], d['1000']['wall_ms_untimed'])"
  done
done
