set -o pipefail
# Round 5: gamma sweep variants (PBH_LIB_VARIANT gs2 / gs8 / gs1k against the default), interleaved,
# then the cfg2 host / kernel profile.
TAG=${1:-r5e}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
for rep in 1 2; do
  for v in default gs2 gs8 gs1k; do
    if [ $v = default ]; then unset PBH_LIB_VARIANT; else export PBH_LIB_VARIANT=$v; fi
    timeout -k 10 200 python tools/ppf_sweep.py > gpurun_out/$TAG/sweep_${v}_$rep.json 2>&1 || exit 1
    echo "$rep $v $(python3 -c "import json,sys; d=json.load(open('gpurun_out/$TAG/sweep_${v}_$rep.json')); print({k: v['ms'] for k, v in d['per_dist'].items() if 'gamma' in k})" 2>/dev/null)"
  done
done
unset PBH_LIB_VARIANT
timeout -k 10 300 python -u tools/profile_cfg2.py 20 > gpurun_out/${TAG}_cfg2_profile.txt 2>&1
echo "profile exit $?"; head -60 gpurun_out/${TAG}_cfg2_profile.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_dists.py tests/test_gpu_ppf.py -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
echo "pytest exit $?"; tail -2 gpurun_out/${TAG}_tests.log; grep -E "^FAILED" gpurun_out/${TAG}_tests.log | head
timeout -k 10 300 python -u tools/ext_sweep.py > gpurun_out/${TAG}_ext_sweep.json 2>&1; echo "ext exit $?"; cat gpurun_out/${TAG}_ext_sweep.json | head -40
