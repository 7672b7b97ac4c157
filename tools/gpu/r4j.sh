set -o pipefail
# Round 4: norm / lognorm placement with the per-wave tail stack (k_place_gen_w).  Generated-column,
# IC and distributed tests, then the A/B against the block-wide queue (PBH_PLACE_WAVE=0).
TAG=${1:-r4j}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ic.py tests/test_gpu_distributed.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_PLACE_WAVE=0" || exit $?
