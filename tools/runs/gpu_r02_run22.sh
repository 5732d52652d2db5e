set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/split_share.py --ns 8,4,2,1 --modes plain,split --knobs 1:65552,1:65537,320:65552 > gpurun_out/r02_run22.log 2>&1
