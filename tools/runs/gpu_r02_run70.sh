# round-2 run 70: the bench multirank tests, including the new one-GPU stream-ordered gather test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_multirank.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_run70_tests.log 2>&1 || exit 1
