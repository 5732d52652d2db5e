# round-2 run 33: tree check after the container re-creation: full -m gpu suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run33_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run33_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 20 > gpurun_out/r02_run33_default.json 2> gpurun_out/r02_run33_default.err || exit 1
