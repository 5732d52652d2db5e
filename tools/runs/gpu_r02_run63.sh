# round-2 run 63: the gather's cross-stream wait shares a hardware queue with the render stream (4 HW queues per
# process), which holds launch k+2 behind launch k+1 (trace of run 59). A/B: GPU_MAX_HW_QUEUES 4 (default) vs 8
# on one GPU's C3 shares through the gather step, plus the default C2 bench under 8 queues
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for n in 2 4 8; do
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run63_q4_share${n}_$r.json 2> gpurun_out/r02_run63_q4_share${n}_$r.err || exit 1
    GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run63_q8_share${n}_$r.json 2> gpurun_out/r02_run63_q8_share${n}_$r.err || exit 1
  done
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run63_q8_c2.json 2> gpurun_out/r02_run63_q8_c2.err || exit 1
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run63_q4_c2.json 2> gpurun_out/r02_run63_q4_c2.err || exit 1
