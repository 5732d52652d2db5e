# round-2 run 56: frame copies that keep launches overlapped (two frame buffers): the new overlap test, the
# full -m gpu suite, smoke, the default bench, the self-gather path at N = 1 (against run 45's 1.569 ms/step),
# a 2-rank gloo rehearsal of the C3 path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_run56_overlap.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run56_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run56_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_run56_default.json 2> gpurun_out/r02_run56_default.err || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --self-gather --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run56_selfgather_$r.json 2> gpurun_out/r02_run56_selfgather_$r.err || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --one-device --steps 5 --warmup 2 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run56_g2.json 2> gpurun_out/r02_run56_g2.err || exit 1
