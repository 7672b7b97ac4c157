set -o pipefail
# Round 4: step-4 parity with the finish class sub-ranges, the scores microbenchmark counters, the
# A/B (finish classes, step-3 NT), PMC traffic of one step, the kernel timeline.
TAG=${1:-r4e}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_dists.py tests/test_gpu_step4_gen.py tests/test_gpu_ic.py tests/test_gpu_scale.py tests/test_gpu_distributed.py tests/test_gpu_step4_buckets.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -40; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_FINISH_CLASSES=0" "PBH_APPLY_NT=1" || exit $?
bash tools/gpu/pmc.sh $TAG || exit $?
python3 -c "
import json; d=json.load(open('gpurun_out/pmc_${TAG}_summary.json'))
for k in ('k_finish_q<1024, 512, false>', 'k_msd1x<1024, 8>', 'k_msd2x<1024, 8>', 'k_place_msdo', 'k_apply_mfma_w2<false>', 'k_place_gen_poisson<false>'):
    v = d.get(k)
    if v: print(k, v['hbm_bytes'], v['dispatches'])
"
timeout -k 10 120 tools/gpu/mbfeistel > gpurun_out/mbfeistel_$TAG.json 2>&1; echo "mbfeistel exit $?"; cat gpurun_out/mbfeistel_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/$TAG/p1 -o pmc --output-format csv -- $R/tools/gpu/mbfeistel > $R/gpurun_out/$TAG/p1.log 2>&1
echo "pmc1 exit $?"
cd $R
bash tools/gpu/timeline.sh ${TAG}_tl > gpurun_out/${TAG}_timeline.txt 2>&1; echo "timeline exit $?"; tail -22 gpurun_out/${TAG}_timeline.txt
timeout -k 10 300 python tools/ext_sweep.py 10000000 > gpurun_out/${TAG}_ext_sweep.json 2>&1; echo "ext_sweep exit $?"; cat gpurun_out/${TAG}_ext_sweep.json | tail -3
