set -o pipefail
# The rocprofv3 one-stream kernel statistics, PMC traffic and VALU passes at HEAD (the GPU tests
# and the bench line ran in the call before).  TAG as $1.
TAG=${1:-r4y}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
cd $R
bash tools/gpu/pmc.sh $TAG || exit $?
bash tools/gpu/pmc_valu.sh ${TAG}_valu || exit $?
