set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/split_share.py --ns 8,4,2,1 --knobs 8:16,16:1 --out gpurun_out/r02_split_share_v4.json > gpurun_out/r02_run7_share.log 2>&1 && \
timeout -k 10 300 python -u tools/split_share.py --stats --ns 8 --out gpurun_out/r02_split_timeline_v2.json > gpurun_out/r02_run7_tl.log 2>&1
