# round-1 GPU run 25: exact BVH for secondary rays: full GPU suite, C4/C5 A/B (BVH vs brute force), bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t25.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t25.log; exit 1; }
tail -2 gpurun_out/t25.log
timeout -k 10 300 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --crop 0,3840,0,54,40 --variants "default=2863,-bvh=815" --out gpurun_out/ab25_c5_bvh.json > gpurun_out/ab25_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab25_c5.log; exit 1; }
cat gpurun_out/ab25_c5.log | tail -5
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r25_bench.json 2> gpurun_out/r25_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r25_bench.err; exit 1; }
cat gpurun_out/r25_bench.json
echo DONE
