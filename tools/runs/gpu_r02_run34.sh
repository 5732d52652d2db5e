# round-2 run 34: chain-parallel pixels (IQPT_SPLIT_CHAIN): parity tests, then the N = 1/2/4/8 share emulation
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_run34_chain_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/split_share.py --modes plain,split,chain --chain-waves 4,16 --out gpurun_out/r02_run34_share.json > gpurun_out/r02_run34_share.log 2>&1 || exit 1
