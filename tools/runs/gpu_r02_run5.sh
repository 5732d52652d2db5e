set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run5_split.log 2>&1 && \
timeout -k 10 400 python -u tools/split_share.py --ns 8,4,2,1 --knobs 8:8,8:16,16:1,16:16,32:16 --out gpurun_out/r02_split_share_v3.json > gpurun_out/r02_run5_share.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02_prof5_share8 -o share8 -- python3 tools/split_share.py --ns 8 --launches 4 --modes split > gpurun_out/r02_run5_prof.log 2>&1
