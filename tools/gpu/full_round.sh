set -o pipefail
# One GPU round: smoke, GPU tests, ppf microbench, bench, a 2-rank sharded rehearsal on the one
# GPU (gloo staging), rocprofv3 kernel stats.
# Ordinary failures (exit 1) continue to the next step; a crash, abort or time limit ends the script.
TAG=${1:-rX}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {  # $1 = exit status, $2 = step name
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1
stop_if_crashed $? smoke
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --maxfail=30 -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
timeout -k 10 300 python tools/microbench_ppf.py > gpurun_out/${TAG}_micro.json 2> gpurun_out/${TAG}_micro.err || exit 1
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
PBH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 --rows 20000000 > gpurun_out/${TAG}_bench2_gloo.json 2> gpurun_out/${TAG}_bench2_gloo.err
stop_if_crashed $? bench2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
