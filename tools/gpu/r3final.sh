set -o pipefail
# Round-3 evidence: every GPU test, the full bench line (e2e, CPU baseline, ppf sweep, copy
# ceiling), the rocprofv3 1-stream kernel stats matching the bench's standalone pass, and the
# PMC traffic passes.  Each GPU step has its own time limit; the script stops at the first failure.
# Usage: bash tools/gpu/r3final.sh TAG [skip-tests]
TAG=${1:-r3final}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 900 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 - <<PY
import json
d=json.load(open("gpurun_out/${TAG}_bench.json"))
print("value", d["value"], "ms", d["ms_per_step"])
print("roofline", json.dumps(d["roofline"]))
print("copy", d["hbm_copy_peak"]["GBps"], "e2e", d["end_to_end"]["value"], d["end_to_end"]["d2h_GBps"])
print("sweep", d["ppf_sweep"]["achieved"], d["ppf_sweep"]["frac"], "cpu", d["cpu_baseline"]["value"])
for k,v in sorted(d["kernels_standalone"].items(), key=lambda kv:-kv[1]["total_ms_per_step"]):
    print(f"  {k:22s} {v['total_ms_per_step']:8.3f} {v['launches']:4d} {v['avg_ms']:.4f} {v['GBps']}")
PY
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 PBH_DEFER_COUNTS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
bash $R/tools/gpu/pmc.sh $TAG || exit $?
if [ "$3" == "full" ]; then
  cd $R
  timeout -k 10 300 python tools/bench_configs.py > gpurun_out/${TAG}_configs.json 2> gpurun_out/${TAG}_configs.err
  rc=$?; echo "configs exit $rc"; [ $rc -eq 0 ] || exit $rc
  bash $R/tools/gpu/pmc_valu.sh ${TAG}_valu
fi
