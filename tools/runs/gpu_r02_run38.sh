# round-2 run 38: chain kernel with 4 lanes per pixel vs 8; parity tests first
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run38_chain_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain --chain-waves 16,16l4,8l4,16l4a --out gpurun_out/r02_run38_share.json > gpurun_out/r02_run38_share.log 2>&1 || exit 1
