set -o pipefail
# Round 4 evidence at HEAD: key GPU tests, the bench line, the rocprofv3 one-stream kernel stats
# (certificate path as in the bench), PMC traffic and VALU passes.  TAG as $1.
TAG=${1:-r4g}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ic.py tests/test_gpu_step4_gen.py tests/test_gpu_scale.py tests/test_gpu_certificate.py tests/test_gpu_distributed.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench exit $rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/show_bench.py gpurun_out/${TAG}_bench.json | head -22
cd /tmp && export TMPDIR=/tmp
PBH_STEP4_STREAMS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG}_1s -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu --no-e2e --ppf-rows 0 > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
cd $R
bash tools/gpu/pmc.sh $TAG || exit $?
bash tools/gpu/pmc_valu.sh ${TAG}_valu || exit $?
