# round-2 run 29: overlap probe (two contexts on two streams vs one) on C2 and C4
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/overlap_probe.py c2 gpurun_out/r02_overlap_c2.json > gpurun_out/r02_run29.log 2>&1
