# round-2 run 66: chain launches with the chain kernel first on the context stream and the anchored kernel on
# stream2, queue counters in two sets zeroed off the critical path: chain/split/overlap tests, then A/B of one
# GPU's C3 N = 4 / 8 shares through the gather step against a library built with -DIQPT_CHAIN_OLD_STREAMS
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_split.py tests/test_gpu_overlap.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_run66_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in 4 8; do
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run66_new_share${n}_$r.json 2> gpurun_out/r02_run66_new_share${n}_$r.err || exit 1
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline --lib tools/libiqpt_oldstreams.so > gpurun_out/r02_run66_old_share${n}_$r.json 2> gpurun_out/r02_run66_old_share${n}_$r.err || exit 1
  done
done
