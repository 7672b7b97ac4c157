set -o pipefail
# Full GPU suite, the N=1e8 all-column step-4 gate, the bench line, then the VALU counter passes.
TAG=${1:-r02b}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
stop_if_crashed() {
  echo "$2 exit $1"
  if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "stopping after $2 (status $1)"; exit "$1"; fi
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
stop_if_crashed $? pytest
tail -6 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u tools/parity_1e8.py --out gpurun_out/${TAG}_parity_1e8.json > gpurun_out/${TAG}_parity_1e8.log 2>&1
stop_if_crashed $? parity
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
stop_if_crashed $? bench
timeout -k 10 200 python -u tools/dag_bench.py > gpurun_out/${TAG}_dag.json 2> gpurun_out/${TAG}_dag.err
stop_if_crashed $? dag_bench
bash tools/gpu/pmc_valu.sh ${TAG}_valu
