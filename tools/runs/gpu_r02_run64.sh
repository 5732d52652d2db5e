# round-2 run 64: bench.py now sets 8 hardware queues itself on the gather path: shares N = 2/4/8 through the
# gather step (no env override), the default C2 bench, a 2-rank gloo rehearsal, the bench multirank test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 2 4 8; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run64_share$n.json 2> gpurun_out/r02_run64_share$n.err || exit 1
done
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run64_c2.json 2> gpurun_out/r02_run64_c2.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --one-device --steps 5 --warmup 2 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run64_g2.json 2> gpurun_out/r02_run64_g2.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_multirank.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run64_tests.log 2>&1 || exit 1
