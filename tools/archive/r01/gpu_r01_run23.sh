# round-1 GPU run 23: tile-major pixel storage: tests, bench, PMC traffic, C3 shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t23.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t23.log; exit 1; }
tail -2 gpurun_out/t23.log
timeout -k 10 400 python bench.py > gpurun_out/r23_bench.json 2> gpurun_out/r23_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r23_bench.err; exit 1; }
cat gpurun_out/r23_bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc23_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc23_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc23_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc23_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc23_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc23_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof23 -o run --output-format csv -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/r23_prof.json 2> gpurun_out/r23_prof.err || { echo PROF_FAILED; tail -20 gpurun_out/r23_prof.err; exit 1; }
cat gpurun_out/r23_prof.json
echo DONE
