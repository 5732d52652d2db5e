# round-2 run 71: chain kernel steps the next slot's state on from the traced state (2 (kL - nsl) draws)
# instead of from the slot's start (2 kL draws): chain/split tests, then A/B of one GPU's C3 N = 4 / 8 shares
# through the gather step against a library built with -DIQPT_CHAIN_STEP_FROM_START, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_run71_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in 4 8; do
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run71_new_share${n}_$r.json 2> gpurun_out/r02_run71_new_share${n}_$r.err || exit 1
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline --lib tools/libiqpt_stepstart.so > gpurun_out/r02_run71_old_share${n}_$r.json 2> gpurun_out/r02_run71_old_share${n}_$r.err || exit 1
  done
done
