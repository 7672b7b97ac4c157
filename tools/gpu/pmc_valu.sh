set -o pipefail
# Issue-level counters (VALU activity, instruction mix) for the VALU-bound kernels: one bench
# step (the IC kernels and the ppf sweep) and one fused / one per-node cfg5 call.  Counter
# passes are separate runs within the gfx950 slot limits (8 SQ, 2 GRBM per pass); counters
# this rocprofv3 does not list are dropped from the pass.
# Usage: bash tools/gpu/pmc_valu.sh TAG [ROWS]
TAG=${1:-valu}
ROWS=${2:-100000000}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
echo "list exit $?"
have() { grep -qw "$1" $OUT/counters_list.txt; }
pick() { local out=""; for c in "$@"; do if have $c; then out="$out $c"; fi; done; echo $out; }
P1=$(pick SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE)
echo "pass1: $P1"; echo "pass2: $P2"
run() {  # name, counters, program...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/$name -o pmc --output-format csv -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name exit $rc"; return $rc
}
run bench_p1 "$P1" python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --rows $ROWS || exit $?
run bench_p2 "$P2" python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --no-e2e --rows $ROWS || exit $?
run dag_p1 "$P1" python3 $R/tools/dag_bench.py --steps 1 --rows $ROWS || exit $?
run dag_p2 "$P2" python3 $R/tools/dag_bench.py --steps 1 --rows $ROWS || exit $?
PBH_DAG=0 run pernode_p1 "$P1" python3 $R/tools/dag_bench.py --steps 1 --rows $ROWS || exit $?
python3 $R/tools/pmc_valu_summary.py $OUT > $R/gpurun_out/${TAG}_summary.json
echo "summary exit $?"
