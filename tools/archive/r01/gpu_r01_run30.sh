# round-1 GPU run 30: running-mean term behind a real branch
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t30.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t30.log; exit 1; }
tail -2 gpurun_out/t30.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r30_bench.json 2> gpurun_out/r30_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r30_bench.err; exit 1; }
cat gpurun_out/r30_bench.json
echo DONE
