# round-2 run 68: one GPU's C3 N = 2 share through the gather step: chain launches (new stream order) against
# the AUTO plain overlapped launches, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of 2 --split chain --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run68_chain_$r.json 2> gpurun_out/r02_run68_chain_$r.err || exit 1
  timeout -k 10 200 python3 bench.py --self-gather --share-of 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run68_auto_$r.json 2> gpurun_out/r02_run68_auto_$r.err || exit 1
done
