set -o pipefail
# Step-4 iteration with A/B: the step-4 / IC / ppf / modeling GPU tests, one bench line per
# setting ("-" = default env), then rocprofv3 kernel stats of the default on one step-4 stream.
# Usage: bash tools/gpu/s4ab.sh TAG "ENV_A" "ENV_B" ...
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ppf.py tests/test_gpu_ic.py tests/test_gpu_modeling.py tests/test_gpu_step4_buckets.py tests/test_gpu_qmc.py ${EXTRA_TESTS} -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
i=0
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.err
  rc=$?; echo "ab$i [$E] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/show_bench.py gpurun_out/${TAG}_ab$i.json > gpurun_out/${TAG}_ab$i.txt
  head -12 gpurun_out/${TAG}_ab$i.txt
  i=$((i+1))
done
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
if [ -n "$PROF2_ENV" ]; then
  env PBH_STEP4_STREAMS=1 $PROF2_ENV timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_2 -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof2_bench.json 2> $R/gpurun_out/${TAG}_prof2.err
  echo "prof2 exit $?"
fi
timeout -k 10 300 python -u $R/tools/ppf_sweep.py > $R/gpurun_out/${TAG}_sweep.json 2> $R/gpurun_out/${TAG}_sweep.err
echo "sweep exit $?"
PBH_LIB_VARIANT=${SWEEP_VARIANT:-} timeout -k 10 300 python -u $R/tools/ppf_sweep.py > $R/gpurun_out/${TAG}_sweep_v.json 2> $R/gpurun_out/${TAG}_sweep_v.err
echo "sweep variant exit $?"
