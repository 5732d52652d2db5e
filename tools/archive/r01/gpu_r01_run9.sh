set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t9.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t9.log; exit 1; }
tail -2 gpurun_out/t9.log
timeout -k 10 300 python bench.py > gpurun_out/bench9.json 2> gpurun_out/bench9.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench9.err; exit 1; }
cat gpurun_out/bench9.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof9.json 2> gpurun_out/prof9.err || { echo PROF_FAILED; tail -20 gpurun_out/prof9.err; exit 1; }
cat gpurun_out/prof9/run_kernel_stats.csv
