# round-1 GPU run 90: end-of-round confirmation on the final tree (leaf sizes as build knobs, interval
# helper added): full GPU suite + smoke, C2 default bench (CPU baseline), rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t90.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t90.log; exit 1; }
tail -1 gpurun_out/t90.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke90.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke90.log; exit 1; }
tail -1 gpurun_out/smoke90.log
timeout -k 10 400 python3 bench.py > gpurun_out/b90_c2.json 2> gpurun_out/b90_c2.err || { echo BENCH_FAILED; tail -20 gpurun_out/b90_c2.err; exit 1; }
cat gpurun_out/b90_c2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p90_stats -o run -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/p90_stats_bench.json 2> gpurun_out/p90_stats_bench.err || { echo PROF_FAILED; tail -20 gpurun_out/p90_stats_bench.err; exit 1; }
cat gpurun_out/p90_stats_bench.json
echo DONE
