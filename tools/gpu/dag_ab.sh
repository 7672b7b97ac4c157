set -o pipefail
# A/B of the fused-graph kernel variants (PBH_LIB_VARIANT) and the per-node path on cfg5.
TAG=${1:-dagab}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
: > gpurun_out/${TAG}.jsonl
for V in "" w3i4 w4i4 w0i8 w3i8; do
  PBH_LIB_VARIANT=$V timeout -k 10 120 python -u tools/dag_bench.py >> gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}_$V.err
  st=$?; echo "variant '$V' exit $st"; [ $st -eq 0 ] || exit $st
done
PBH_DAG=0 timeout -k 10 120 python -u tools/dag_bench.py >> gpurun_out/${TAG}.jsonl 2> gpurun_out/${TAG}_pernode.err
st=$?; echo "per-node exit $st"; [ $st -eq 0 ] || exit $st
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_modeling.py -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
st=$?; tail -5 gpurun_out/${TAG}_tests.log; echo "pytest exit $st"; exit $st
