set -o pipefail
# HBM traffic of every kernel of one bench step (rocprofv3 PMC), one counter per pass as the
# MI355X guide prescribes (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: separate runs).
# Usage: bash tools/gpu/pmc.sh TAG [ROWS]
TAG=${1:-rX}
ROWS=${2:-100000000}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex 'pbh' -d $R/gpurun_out/pmc_${TAG}_$C -o pmc \
    --output-format csv -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu --rows $ROWS \
    > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1
  rc=$?
  echo "pmc $C exit $rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_${TAG}_FETCH_SIZE $R/gpurun_out/pmc_${TAG}_WRITE_SIZE \
  > $R/gpurun_out/pmc_${TAG}_summary.json
