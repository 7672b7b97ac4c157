set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -v -s -rf --timeout 1200 --timeout-method thread -p no:cacheprovider -k gate > gpurun_out/r3h_tests.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/r3h_tests.log
bash tools/gpu/ab3.sh ab4 "PBH_CERT=1" "PBH_CERT=0" || exit $?
timeout -k 10 600 python bench.py > gpurun_out/r3h_bench.json 2> gpurun_out/r3h_bench.err; echo "bench exit $?"
python3 -c "
import json; d=json.load(open('gpurun_out/r3h_bench.json'))
print(d['value'], d['ms_per_step'], json.dumps(d['end_to_end']), d['roofline']['kernel'], d['roofline']['frac'])
for k,v in sorted(d['kernels_standalone'].items(), key=lambda kv:-kv[1]['total_ms_per_step']): print('  ', k, v['total_ms_per_step'], v['launches'])
"
