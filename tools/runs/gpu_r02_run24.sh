# round-2 run 24 (session 4 start): full -m gpu suite, smoke, default bench line on the restored tree
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run24_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run24_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r02_run24_default.json 2> gpurun_out/r02_run24_default.err || exit 1
