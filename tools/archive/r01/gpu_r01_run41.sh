# round-1 GPU run 41: full-frame parity (C2 at bench size, C4 one pass, C5 band)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_fullframe.py -x -q -m gpu --durations=0 > gpurun_out/t41.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t41.log; exit 1; }
tail -8 gpurun_out/t41.log
echo DONE
