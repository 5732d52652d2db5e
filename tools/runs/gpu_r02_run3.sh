set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run3_split.log 2>&1 && \
timeout -k 10 300 python -u tools/split_share.py --out gpurun_out/r02_split_share_v2.json > gpurun_out/r02_run3_share.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_prof_share8 -o share8 -- python3 tools/split_share.py --ns 8 --launches 5 > gpurun_out/r02_run3_prof.log 2>&1
