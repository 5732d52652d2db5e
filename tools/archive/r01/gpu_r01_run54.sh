# round-1 GPU run 54: camera tests (opt-in axis variant), materials, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py tests/test_gpu_materials.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t54.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t54.log; exit 1; }
tail -2 gpurun_out/t54.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/b54.json 2> gpurun_out/b54.err || { echo BENCH_FAILED; tail -30 gpurun_out/b54.err; exit 1; }
cat gpurun_out/b54.json
echo DONE
