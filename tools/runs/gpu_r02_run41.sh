# round-2 run 41: chain kernel with a wave-level pending-pixel queue filled in batches of 8 (one fetch stage per iteration)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run41_chain_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --chain-waves 16l4,16a,16l4a --out gpurun_out/r02_run41_share.json > gpurun_out/r02_run41_share.log 2>&1 || exit 1
