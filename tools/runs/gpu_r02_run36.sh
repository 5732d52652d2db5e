# round-2 run 36: chain launches with every tile in the chain kernel ("a" rows) vs split-set only, N = 1/2/4/8
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --chain-waves 16,8a,16a,32a --out gpurun_out/r02_run36_share.json > gpurun_out/r02_run36_share.log 2>&1 || exit 1
