# round-2 run 44: kOptCamAxis on overlapped launches by default: full -m gpu suite, smoke, default bench; chain shares
# with the short camera (--opt: plain and chain kernels both take it)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run44_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run44_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 20 > gpurun_out/r02_run44_default.json 2> gpurun_out/r02_run44_default.err || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --ns 1,2,4,8 --opt 0x44b2f --out gpurun_out/r02_run44_share_camaxis.json > gpurun_out/r02_run44_share_camaxis.log 2>&1 || exit 1
