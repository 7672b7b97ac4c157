set -o pipefail
# Interleaved A/B: the default library against build variant $1 (build.py --variant): the ppf sweep
# and a 5-step bench per run, two rounds.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do
  for v in default $1; do
    if [ $v = default ]; then unset PBH_LIB_VARIANT; else export PBH_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/ppf_sweep.py > gpurun_out/abv_sweep_${v}_$rep.json 2>&1 || exit 1
    timeout -k 10 300 python bench.py --no-cpu --no-e2e --ppf-rows 0 --steps 5 > gpurun_out/abv_bench_${v}_$rep.json 2> gpurun_out/abv_bench_${v}_$rep.err || exit 1
    echo "$rep $v done"
  done
done
