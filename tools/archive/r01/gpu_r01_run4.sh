set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t4.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t4.log; exit 1; }
tail -2 gpurun_out/t4.log
timeout -k 10 600 python tools/ab_kernel.py --config c2 --rounds 7 --out gpurun_out/ab4.json > gpurun_out/ab4.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab4.log; exit 1; }
cat gpurun_out/ab4.json
