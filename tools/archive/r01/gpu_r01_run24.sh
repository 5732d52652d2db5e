# round-1 GPU run 24: material table kernel variant: full GPU suite + bench (default path unchanged)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t24.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t24.log; exit 1; }
tail -2 gpurun_out/t24.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r24_bench.json 2> gpurun_out/r24_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r24_bench.err; exit 1; }
cat gpurun_out/r24_bench.json
echo DONE
