set -o pipefail
# Round 5: setup-table cache: dist / ppf / modeling / step-4 tests, cfg2 profile, bench.
TAG=${1:-r5l}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 700 python -u -m pytest tests/test_gpu_dists.py tests/test_gpu_ppf.py tests/test_gpu_modeling.py tests/test_gpu_step4_gen.py tests/test_gpu_tables.py tests/test_gpu_dag.py -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -3 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|error|FAIL" gpurun_out/$TAG/tests.log | head -30; exit 1; }
timeout -k 10 300 python -u tools/profile_cfg2.py 20 > gpurun_out/$TAG/cfg2_profile.txt 2>&1; echo "profile $?"; head -24 gpurun_out/$TAG/cfg2_profile.txt
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['reference_stream']['value'], d['roofline']['frac'], d['ppf_sweep']['frac'])"
