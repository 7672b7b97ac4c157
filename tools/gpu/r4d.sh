set -o pipefail
# Round 4: the scores microbenchmark with instruction counters, then W2 against W2+NT (interleaved).
TAG=${1:-r4d}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 120 tools/gpu/mbfeistel > gpurun_out/mbfeistel_$TAG.json 2>&1; echo "mbfeistel exit $?"; cat gpurun_out/mbfeistel_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE -d $R/gpurun_out/$TAG/p1 -o pmc --output-format csv -- $R/tools/gpu/mbfeistel > $R/gpurun_out/$TAG/p1.log 2>&1
echo "pmc1 exit $?"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $R/gpurun_out/$TAG/p2 -o pmc --output-format csv -- $R/tools/gpu/mbfeistel > $R/gpurun_out/$TAG/p2.log 2>&1
echo "pmc2 exit $?"
cd $R
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_APPLY_NT=1"
bash $R/tools/gpu/timeline.sh ${TAG}_tl > $R/gpurun_out/${TAG}_timeline.txt 2>&1; echo "timeline exit $?"; tail -25 $R/gpurun_out/${TAG}_timeline.txt
