set -o pipefail
# Round 6: cfg2 / cfg5 side measurements (tools/bench_configs.py) and cfg2's host overhead at 1e3 / 1e7
TAG=${1:-r6cfg}
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u tools/bench_configs.py --steps 3 > gpurun_out/$TAG/configs.json 2> gpurun_out/$TAG/configs.err || { tail -20 gpurun_out/$TAG/configs.err; exit 1; }
cat gpurun_out/$TAG/configs.json | head -c 3000
for n in 1000 10000000; do
  timeout -k 10 300 python3 -u tools/cfg2_overhead.py $n 200 > gpurun_out/$TAG/cfg2_overhead_$n.json 2> gpurun_out/$TAG/cfg2_overhead_$n.err || { tail -20 gpurun_out/$TAG/cfg2_overhead_$n.err; exit 1; }
  tail -c 600 gpurun_out/$TAG/cfg2_overhead_$n.json
done
