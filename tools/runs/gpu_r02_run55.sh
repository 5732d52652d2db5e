# round-2 run 55: tree check after container re-creation: full -m gpu suite, smoke, the default bench exactly as the driver runs it
# (60-s CPU baseline), a 2-rank gloo rehearsal of the C3 path
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run55_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run55_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_run55_default.json 2> gpurun_out/r02_run55_default.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --one-device --steps 5 --warmup 2 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run55_g2.json 2> gpurun_out/r02_run55_g2.err || exit 1
