set -o pipefail
# Round 4 final evidence at HEAD: every GPU test, the bench line, the rocprofv3 one-stream kernel
# statistics, PMC traffic and VALU passes.  TAG as $1.
TAG=${1:-r4z}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_show.txt; head -22 gpurun_out/${TAG}_show.txt
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
cd $R
bash tools/gpu/pmc.sh $TAG || exit $?
bash tools/gpu/pmc_valu.sh ${TAG}_valu || exit $?
