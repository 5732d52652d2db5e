# round-2 run 28: C2 wave timeline with each wave's first queue position (tail analysis)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_kernel.py --config c2 --rounds 3 --variants default=396079 --stats-opt 396079 --timeline-npy gpurun_out/r02_c2_timeline.npy --out gpurun_out/r02_c2_timeline.json > gpurun_out/r02_run28.log 2>&1
