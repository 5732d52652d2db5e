set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/split_share.py --ns 8,1 --modes plain --knobs 65535:1,65535:16,600:16 --out gpurun_out/r02_split_share_v7.json > gpurun_out/r02_run15_share.log 2>&1 && \
timeout -k 10 300 python -u tools/split_share.py --stats --ns 8 --out gpurun_out/r02_split_timeline_v4.json > gpurun_out/r02_run15_tl.log 2>&1
