# round-2 run 39: chain defaults (16 waves/CU, AUTO at < 2 pixels per lane): full -m gpu suite, smoke, default bench,
# a 4-rank gloo rehearsal of the C3 path on one GPU, the N = 1/2/4/8 share table with AUTO
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run39_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run39_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --cpu-seconds 20 > gpurun_out/r02_run39_default.json 2> gpurun_out/r02_run39_default.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 4 --backend gloo --one-device --steps 5 --warmup 2 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run39_g4_rehearsal.json 2> gpurun_out/r02_run39_g4_rehearsal.err || exit 1
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --out gpurun_out/r02_run39_share.json > gpurun_out/r02_run39_share.log 2>&1 || exit 1
