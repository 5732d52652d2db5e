# round-1 GPU run 60: C5 and C4 bench lines after the sphere BVH
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/b60_c5.json 2> gpurun_out/b60_c5.err || { echo BENCH5_FAILED; tail -30 gpurun_out/b60_c5.err; exit 1; }
cat gpurun_out/b60_c5.json
timeout -k 10 400 python bench.py --config c4 --spp 16 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/b60_c4.json 2> gpurun_out/b60_c4.err || { echo BENCH4_FAILED; tail -30 gpurun_out/b60_c4.err; exit 1; }
cat gpurun_out/b60_c4.json
echo DONE
