set -o pipefail
# Round 5: the round-5 distributions, the poisson tests, then the N=1e8 gate against the reference's
# own steps 1-2 (records/parity_1e8_reference_steps.json).
TAG=${1:-r5c}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_dists.py tests/test_gpu_ppf.py tests/test_gpu_step4_gen.py tests/test_gpu_distributed.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
timeout -k 10 1000 python -u -m pytest "tests/test_gpu_scale.py::test_cfg3_step4_gate_1e8_reference_steps_1_2" -m gpu -q -s -rf --timeout 960 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gate.log 2>&1
rc=$?; echo "gate exit $rc"; tail -5 gpurun_out/${TAG}_gate.log
