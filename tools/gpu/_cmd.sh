set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_step4_gen.py tests/test_gpu_ppf.py tests/test_gpu_ic.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/s4c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/s4c_tests.log; [ $rc -gt 1 ] && exit $rc
for V in default w2 w0; do
  if [ $V = default ]; then unset PBH_LIB_VARIANT; else export PBH_LIB_VARIANT=$V; fi
  PBH_STEP4_STREAMS=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/s4c_$V.json 2>/dev/null || exit $?
  echo "== $V (1 stream)"; python3 tools/show_bench.py gpurun_out/s4c_$V.json | head -12
done
unset PBH_LIB_VARIANT
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --no-e2e --ppf-rows 0 > gpurun_out/s4c_2s.json 2>/dev/null && echo "== default 2 streams" && python3 tools/show_bench.py gpurun_out/s4c_2s.json | head -3
