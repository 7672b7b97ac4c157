set -o pipefail
# Round-end evidence: the full GPU suite, the N=1e8 all-column step-4 gate, the bench line
# (e2e + CPU baseline + ppf sweep), rocprofv3 kernel stats (3 step-4 streams as benched, and one
# stream for standalone durations), FETCH/WRITE PMC passes, the VALU counter passes, cfg2 / cfg5
# side measurements and the CPU baseline at 1e6 / 1e7.  A crash, abort or time limit ends it.
TAG=${1:-fin}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u tools/parity_1e8.py --out gpurun_out/${TAG}_parity_1e8.json > gpurun_out/${TAG}_parity_1e8.log 2>&1
stop_if_crashed $? parity
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
stop_if_crashed $? bench
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.txt
timeout -k 10 300 python -u tools/bench_configs.py --steps 3 --cpu-n 200000 > gpurun_out/${TAG}_configs.json 2> gpurun_out/${TAG}_configs.err
stop_if_crashed $? configs
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
stop_if_crashed $? prof
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof1s_bench.json 2> $R/gpurun_out/${TAG}_prof1s.err
stop_if_crashed $? prof1s
bash $R/tools/gpu/pmc.sh $TAG
stop_if_crashed $? pmc
bash $R/tools/gpu/pmc_valu.sh ${TAG}_valu
stop_if_crashed $? pmc_valu
cd $R
timeout -k 10 900 python -u tools/cpu_baseline_side.py --rows 1000000 10000000 > gpurun_out/${TAG}_cpu_side.json 2> gpurun_out/${TAG}_cpu_side.err
echo "cpu side exit $?"
