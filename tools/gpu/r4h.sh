set -o pipefail
# Round 4: scores + Gram in one pass (k_scores_gram).  Its parity test and the generated-column /
# IC tests first, then the interleaved A/B against the separate kernels (PBH_SCORES_GRAM=0).
TAG=${1:-r4h}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py -k "scores_gram" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_sg.log 2>&1
rc=$?; echo "sg pytest exit $rc"; tail -8 gpurun_out/${TAG}_sg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ic.py tests/test_gpu_certificate.py -m gpu -q -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head -20; [ $rc -le 1 ] || exit $rc
bash tools/gpu/ab_env.sh ${TAG}_ab "-" "PBH_SCORES_GRAM=0" || exit $?
