set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/split_share.py --stats --ns 8,1 --out gpurun_out/r02_split_timeline_v1.json > gpurun_out/r02_run6.log 2>&1
