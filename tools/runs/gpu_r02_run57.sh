# round-2 run 57: one GPU's C3 shares through the per-step gather path (--share-of N --self-gather), with
# the frame copies that keep launches overlapped; N = 2 also with --overlap off (A/B)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 1 2 4 8; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run57_share$n.json 2> gpurun_out/r02_run57_share$n.err || exit 1
done
timeout -k 10 200 python3 bench.py --self-gather --share-of 2 --overlap off --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run57_share2_ovloff.json 2> gpurun_out/r02_run57_share2_ovloff.err || exit 1
timeout -k 10 200 python3 bench.py --self-gather --share-of 2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run57_share2_b.json 2> gpurun_out/r02_run57_share2_b.err || exit 1
