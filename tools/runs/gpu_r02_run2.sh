set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_run2_split.log 2>&1 && \
timeout -k 10 300 python -u tools/split_share.py --out gpurun_out/r02_split_share_v1.json > gpurun_out/r02_run2_share.log 2>&1
