set -o pipefail
# Round 6: rocprofv3 kernel-trace summaries of the headline bench step (bench.py, side figures off):
# one step-4 lane (PBH_STEP4_STREAMS=1: standalone durations) and as benched (three lanes)
TAG=${1:-r6k}
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$TAG
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 --operator-rows 0 --refstream-rows 0"
export PBH_STEP4_STREAMS=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof_1stream -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/$TAG/bench_1stream.json 2> $R/gpurun_out/$TAG/bench_1stream.err || { echo "1stream failed"; tail -20 $R/gpurun_out/$TAG/bench_1stream.err; exit 1; }
unset PBH_STEP4_STREAMS
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof_lanes -o run --output-format csv -- python3 $R/bench.py $ARGS > $R/gpurun_out/$TAG/bench_lanes.json 2> $R/gpurun_out/$TAG/bench_lanes.err || { echo "lanes failed"; tail -20 $R/gpurun_out/$TAG/bench_lanes.err; exit 1; }
find $R/gpurun_out/$TAG -name "*kernel_stats.csv"
