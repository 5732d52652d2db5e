# round-1 GPU run 42: re-validation after the container restore: full GPU suite, smoke, default bench, rocprof stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t42.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t42.log; exit 1; }
tail -3 gpurun_out/t42.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || { echo SMOKE_FAILED; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/b42.json 2> gpurun_out/b42.err || { echo BENCH_FAILED; tail -30 gpurun_out/b42.err; exit 1; }
cat gpurun_out/b42.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof42 -o run -- python bench.py --no-cpu-baseline > gpurun_out/b42p.json 2> gpurun_out/b42p.err || { echo PROF_FAILED; tail -30 gpurun_out/b42p.err; exit 1; }
find gpurun_out/prof42 -name "*stats*"
echo DONE
