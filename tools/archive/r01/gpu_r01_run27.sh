# round-1 GPU run 27: camera-ray path chosen by timing (tile masks vs BVH); C4/C5 bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t27.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t27.log; exit 1; }
tail -2 gpurun_out/t27.log
timeout -k 10 400 python bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r27_bench_c5.json 2> gpurun_out/r27_bench_c5.err || { echo BENCH5_FAILED; tail -30 gpurun_out/r27_bench_c5.err; exit 1; }
cat gpurun_out/r27_bench_c5.json
timeout -k 10 400 python bench.py --config c4 --spp 16 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r27_bench_c4.json 2> gpurun_out/r27_bench_c4.err || { echo BENCH4_FAILED; tail -30 gpurun_out/r27_bench_c4.err; exit 1; }
cat gpurun_out/r27_bench_c4.json
echo DONE
