# round-2 run 32: overlapped launches (static cost order, one block slot per CU left free): full -m gpu
# suite, smoke, default bench (60-s CPU baseline), rocprofv3 kernel stats of the default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run32_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run32_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r02_run32_default.json 2> gpurun_out/r02_run32_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof32_c2 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/r02_prof32_c2.json 2> gpurun_out/r02_prof32_c2.err || exit 1
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/r02_run32_c4.json 2> gpurun_out/r02_run32_c4.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --spp 16 --steps 5 --no-cpu-baseline --verify-rows 4 > gpurun_out/r02_run32_c5.json 2> gpurun_out/r02_run32_c5.err || exit 1
