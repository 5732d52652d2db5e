# round-2 run 46: short camera wherever it qualifies (plain, overlapped, chain), chain pixel loads in one round trip: full -m gpu suite, smoke, default
# bench, AUTO share table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run46_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run46_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 20 > gpurun_out/r02_run46_default.json 2> gpurun_out/r02_run46_default.err || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --ns 1,2,4,8 --out gpurun_out/r02_run46_share.json > gpurun_out/r02_run46_share.log 2>&1 || exit 1
