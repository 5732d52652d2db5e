# round-1 GPU run 73: 5-wave BVH-primary in production: GPU suite, C5 bench line (timing picks the variant)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t73.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t73.log; exit 1; }
tail -2 gpurun_out/t73.log
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c5.json > gpurun_out/b73_c5.json 2> gpurun_out/b73_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/b73_c5.err; exit 1; }
cat gpurun_out/b73_c5.json
timeout -k 10 400 python3 bench.py --config c4 --spp 16 --steps 5 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c4.json > gpurun_out/b73_c4.json 2> gpurun_out/b73_c4.err || { echo BENCH4_FAILED; tail -20 gpurun_out/b73_c4.err; exit 1; }
cat gpurun_out/b73_c4.json
echo DONE
