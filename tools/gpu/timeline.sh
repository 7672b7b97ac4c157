set -o pipefail
# Kernel timeline of bench steps (rocprofv3 kernel trace, default streams), summarised by
# tools/timeline.py.  Usage: bash tools/gpu/timeline.sh TAG [extra bench args]
TAG=${1:-tl}; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 "$@" > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
rc=$?; echo "prof exit $rc"; [ $rc -eq 0 ] || exit $rc
T=$(find $R/gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python3 $R/tools/timeline.py $T 3
