# round-1 GPU run 3: all gpu tests, smoke, PMC traffic passes for the C2 render kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t3.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t3.log; exit 1; }
tail -3 gpurun_out/t3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke3.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke3.log; exit 1; }
cat gpurun_out/smoke3.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc_write.log; exit 1; }
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv" | head -20
