# round-2 run 40: (rejected) per-walker prefetch of the next pixel, one stage per iteration
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run40_chain_tests.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --chain-waves 16l4,16a,16l4a --out gpurun_out/r02_run40_share.json > gpurun_out/r02_run40_share.log 2>&1 || exit 1
