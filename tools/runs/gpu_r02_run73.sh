# round-2 run 73: frame copies after chain launches on a third stream (the next chain launch writes the other
# frame buffer, the one after waits for the copy): chain/overlap/split/multirank tests, C3 N = 4 / 8 shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_split.py tests/test_gpu_overlap.py tests/test_gpu_bench_multirank.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run73_tests.log 2>&1 || exit 1
for r in 1 2; do
  for n in 4 8; do
    timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run73_share${n}_$r.json 2> gpurun_out/r02_run73_share${n}_$r.err || exit 1
  done
done
