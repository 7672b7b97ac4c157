set -o pipefail
# Interleaved A/B of the ppf sweep: the default library against build variant $1 (build.py --variant)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
  for v in default $1; do
    if [ $v = default ]; then unset PBH_LIB_VARIANT; else export PBH_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/ppf_sweep.py > gpurun_out/absw_${v}_$rep.json 2>&1 || exit 1
  done
done
