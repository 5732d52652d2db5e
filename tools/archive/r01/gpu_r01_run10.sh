set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t10.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t10.log; exit 1; }
tail -2 gpurun_out/t10.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench10.json 2> gpurun_out/bench10.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench10.err; exit 1; }
cat gpurun_out/bench10.json
