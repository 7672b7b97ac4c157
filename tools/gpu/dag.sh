set -o pipefail
# Fused DAG kernel: its GPU tests, then cfg2/cfg5 side measurements fused and per-node.
TAG=${1:-dag}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_dag.py tests/test_gpu_modeling.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
st=$?; tail -5 gpurun_out/${TAG}_tests.log; echo "pytest exit $st"
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
timeout -k 10 300 python -u tools/bench_configs.py --steps 3 --cpu-n 200000 > gpurun_out/${TAG}_cfg_fused.json 2> gpurun_out/${TAG}_cfg_fused.err
st=$?; echo "cfg fused exit $st"; [ $st -eq 0 ] || exit $st
PBH_DAG=0 timeout -k 10 300 python -u tools/bench_configs.py --steps 3 --cpu-n 200000 > gpurun_out/${TAG}_cfg_pernode.json 2> gpurun_out/${TAG}_cfg_pernode.err
st=$?; echo "cfg per-node exit $st"; exit $st
