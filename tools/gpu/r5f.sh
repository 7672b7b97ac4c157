set -o pipefail
# Round 5: grouped native-LHS columns (pbh_lhs_ppf_columns) for cfg2: profile, the dist/modeling
# tests, then a bench line.
TAG=${1:-r5f}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/profile_cfg2.py 20 > gpurun_out/$TAG/cfg2_profile.txt 2>&1 || { echo "profile failed $?"; tail -30 gpurun_out/$TAG/cfg2_profile.txt; exit 1; }
head -60 gpurun_out/$TAG/cfg2_profile.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_dists.py tests/test_gpu_modeling.py tests/test_gpu_dag.py tests/test_gpu_streams.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -3 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; cat gpurun_out/$TAG/bench.json
