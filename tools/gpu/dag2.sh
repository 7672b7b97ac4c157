set -o pipefail
TAG=${1:-dag2}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_modeling.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
st=$?; tail -3 gpurun_out/${TAG}_tests.log; echo "pytest exit $st"; [ $st -eq 0 ] || exit $st
: > gpurun_out/${TAG}.jsonl
for V in "" w4i8; do
  PBH_LIB_VARIANT=$V timeout -k 10 120 python -u tools/dag_bench.py >> gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}_$V.err
  st=$?; echo "variant '$V' exit $st"; [ $st -eq 0 ] || exit $st
done
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-e2e > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
echo "bench exit $?"
