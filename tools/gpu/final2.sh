set -o pipefail
# Final check of the round's build: the full GPU suite, the N=1e8 gate, the bench line (defaults),
# rocprofv3 kernel stats (as benched and on one step-4 stream), the FETCH/WRITE PMC passes, then
# an A/B bench of one setting ($AB_ENV).  A crash, abort or time limit ends it.
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
head -3 gpurun_out/${TAG}_bench.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
stop_if_crashed $? prof
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof1s_bench.json 2> $R/gpurun_out/${TAG}_prof1s.err
stop_if_crashed $? prof1s
bash $R/tools/gpu/pmc.sh $TAG
stop_if_crashed $? pmc
cd $R
if [ -n "$AB_ENV" ]; then
  env $AB_ENV timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err
  stop_if_crashed $? ab
  python3 tools/show_bench.py gpurun_out/${TAG}_ab.json | head -2
fi
