set -o pipefail
# Bench-only A/B: one bench line per setting ("-" = default env), no tests.
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
i=0
for E in "$@"; do
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/${TAG}_ab$i.json 2> gpurun_out/${TAG}_ab$i.err
  rc=$?; echo "ab$i [$E] exit $rc"; [ $rc -eq 0 ] || exit $rc
  python3 tools/show_bench.py gpurun_out/${TAG}_ab$i.json | head -1
  i=$((i+1))
done
