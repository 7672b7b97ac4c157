set -o pipefail
# Round 6: interleaved A/B of the side workloads: bash tools/gpu/r6_ab.sh TAG MODE(--refstream|--operator|'') VARIANTS...
TAG=${1:-r6ab}; MODE=$2; shift 2
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python3 -u tools/ab_step.py --rounds 2 --steps 3 $MODE "$@" > gpurun_out/$TAG/ab.log 2> gpurun_out/$TAG/ab.err; st=$?
cat gpurun_out/$TAG/ab.log | grep variant | grep -v runs; [ $st -eq 0 ] || { tail -20 gpurun_out/$TAG/ab.err; exit 1; }
