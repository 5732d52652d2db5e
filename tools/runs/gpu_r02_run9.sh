set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run9_split.log 2>&1 && \
timeout -k 10 400 python -u tools/split_share.py --ns 8,4,2,1 --knobs 384:1,320:16,512:16,257:16 --out gpurun_out/r02_split_share_v5.json > gpurun_out/r02_run9_share.log 2>&1
