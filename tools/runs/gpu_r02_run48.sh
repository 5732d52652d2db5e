# round-2 run 48: (rejected, reverted) chain list by slots-per-sample threshold, the rest anchored in the plain kernel; C5 line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run48_chain_tests.log 2>&1 || exit 1
timeout -k 10 500 python3 tools/split_share.py --modes plain,chain --ns 2,4,8 --warm 3 --chain-waves 16t320,16t384,16t448,16t512 --out gpurun_out/r02_run48_share.json > gpurun_out/r02_run48_share.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --config c5 --spp 16 --steps 5 --no-cpu-baseline --verify-rows 4 > gpurun_out/r02_run48_c5.json 2> gpurun_out/r02_run48_c5.err || exit 1
