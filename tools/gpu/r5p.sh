set -o pipefail
# Round 5 evidence at HEAD: sharded general correlators (distributed tests), PMC traffic + VALU
# passes of one bench step, rocprof kernel stats (one step-4 stream and as benched).
TAG=${1:-r5p}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q -rf --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests_dist.log 2>&1
st=$?; echo "pytest exit $st"; tail -2 gpurun_out/$TAG/tests_dist.log; [ $st -eq 0 ] || { grep -E "Error|FAIL" gpurun_out/$TAG/tests_dist.log | head -20; exit 1; }
bash tools/gpu/pmc.sh $TAG || exit $?
bash tools/gpu/pmc_valu.sh valu_$TAG || exit $?
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof1s_bench.json 2> $R/gpurun_out/${TAG}_prof1s.err
echo "prof1s exit $?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
cd $R; python3 -c "
import json; d=json.load(open('gpurun_out/pmc_${TAG}_summary.json'))
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get('hbm_bytes', 0))[:12]: print(k, v)
"
