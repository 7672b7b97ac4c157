set -o pipefail
# Round 4, first box: the Feistel microbenchmark, then every GPU test at HEAD.
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 120 tools/gpu/mbfeistel > gpurun_out/mbfeistel_r4a.json 2>&1; echo "mbfeistel exit $?"; cat gpurun_out/mbfeistel_r4a.json
bash tools/gpu/r4tests.sh r4a_tests tests/test_gpu_dists.py tests/test_gpu_modeling.py tests
