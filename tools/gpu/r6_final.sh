set -o pipefail
# Round 6: the bench line, then the HBM traffic and VALU PMC passes of one bench step, at HEAD
R=$GRAFT_REPO_ROOT; cd $R
bash tools/gpu/r6_bench.sh r6fin && bash tools/gpu/pmc.sh r6p && bash tools/gpu/pmc_valu.sh r6v
