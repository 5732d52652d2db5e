# round-2 run 45: share table with the short camera in both kernels (--opt: kOptDefault | kOptCamAxis)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --ns 1,2,4,8 --opt 0x44b2f --out gpurun_out/r02_run45_share_camaxis.json > gpurun_out/r02_run45_share_camaxis.log 2>&1 || exit 1
