set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/split_share.py --ns 8,4 --modes split --opt 35631 > gpurun_out/r02_run20_lb5.log 2>&1 && \
timeout -k 10 300 python -u tools/split_share.py --ns 8,4 --modes plain,split > gpurun_out/r02_run20_lb4.log 2>&1
