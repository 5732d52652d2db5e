# round-2 run 30: overlapped launches (kOptOverlap): overlap tests, parity tests, default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_run30_overlap.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_run30_parity.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r02_run30_default.json 2> gpurun_out/r02_run30_default.err || exit 1
