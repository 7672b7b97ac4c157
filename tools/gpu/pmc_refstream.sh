set -o pipefail
# Issue-level counters of the reference-stream side figure's kernels (one call of
# tools/ref_stream_profile.py at 1e7 x 32): the one-sweep passes, the decode and the scatter.
# Usage: bash tools/gpu/pmc_refstream.sh TAG
TAG=${1:-pmcref}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1
echo "list exit $?"
have() { grep -qw "$1" $OUT/counters_list.txt; }
pick() { local out=""; for c in "$@"; do if have $c; then out="$out $c"; fi; done; echo $out; }
P1=$(pick SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE)
P2=$(pick SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE)
echo "pass1: $P1"; echo "pass2: $P2"
run() {  # name, counters, program...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $OUT/$name -o pmc --output-format csv -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name exit $rc"; return $rc
}
run ref_p1 "$P1" python3 $R/tools/ref_stream_profile.py 1 || exit $?
run ref_p2 "$P2" python3 $R/tools/ref_stream_profile.py 1 || exit $?
python3 $R/tools/pmc_valu_summary.py $OUT > $R/gpurun_out/${TAG}_summary.json
echo "summary exit $?"
