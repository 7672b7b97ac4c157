set -o pipefail
# Round 5: cached graph analysis: modeling / dag / dists / distributed / streams tests, cfg2 profile, bench.
TAG=${1:-r5t}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 900 python -u -m pytest tests/test_gpu_modeling.py tests/test_gpu_dag.py tests/test_gpu_dists.py tests/test_gpu_distributed.py tests/test_gpu_correlators.py tests/test_gpu_streams.py -m gpu -x -q -rf --timeout 500 --timeout-method thread -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
st=$?; echo "pytest exit $st"; tail -2 gpurun_out/$TAG/tests.log; [ $st -eq 0 ] || { grep -E "Error|FAIL" gpurun_out/$TAG/tests.log | head -20; exit 1; }
timeout -k 10 300 python -u tools/cfg2_overhead.py 1000 200 > gpurun_out/$TAG/o1k.json 2>&1; echo "o $?"; tail -1 gpurun_out/$TAG/o1k.json
timeout -k 10 300 python -u tools/profile_cfg2.py 20 > gpurun_out/$TAG/cfg2_profile.txt 2>&1; echo "profile $?"; grep -A3 '"10000000"' gpurun_out/$TAG/cfg2_profile.txt | head -4; grep wall_ms_untimed gpurun_out/$TAG/cfg2_profile.txt
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err; echo "bench exit $?"; python3 -c "
import json; d=json.load(open('gpurun_out/$TAG/bench.json')); print(d['value'], d['ms_per_step'], d['reference_stream']['value'], d['reference_stream']['stream_only'], d['roofline']['frac'], d['ppf_sweep']['frac'])"
