set -o pipefail
TAG=${1:-rX}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/${TAG}_smoke.log 2>&1; echo "smoke exit $?" >> gpurun_out/${TAG}_smoke.log
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --maxfail=30 -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1; echo "pytest exit $?" >> gpurun_out/${TAG}_tests.log
timeout -k 10 300 python tools/microbench_ppf.py > gpurun_out/${TAG}_micro.json 2> gpurun_out/${TAG}_micro.err || exit 1
timeout -k 10 700 python bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${TAG} -o bench --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/${TAG}_prof_bench.json 2> $R/gpurun_out/${TAG}_prof.err
echo "prof exit $?"
