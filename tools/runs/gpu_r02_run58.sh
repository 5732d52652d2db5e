# round-2 run 58: C3 shares N = 4 / 8 through the gather path: plain overlapped launches (--split off) against
# the AUTO chain launches, alternating, two runs each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for n in 4 8; do
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --split off --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run58_share${n}_plain_$r.json 2> gpurun_out/r02_run58_share${n}_plain_$r.err || exit 1
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run58_share${n}_auto_$r.json 2> gpurun_out/r02_run58_share${n}_auto_$r.err || exit 1
  done
done
