# round-2 run 74: final-tree check (library rebuilt after the second rejected A/B): full -m gpu suite, smoke, the default bench as the driver
# runs it (60-s CPU baseline), one GPU's C3 shares N = 2/4/8 through the gather step, a 2-rank gloo rehearsal
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run74_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run74_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r02_run74_default.json 2> gpurun_out/r02_run74_default.err || exit 1
for n in 2 4 8; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run74_share$n.json 2> gpurun_out/r02_run74_share$n.err || exit 1
done
timeout -k 10 300 python3 bench.py --gpus 2 --backend gloo --one-device --steps 5 --warmup 2 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run74_g2.json 2> gpurun_out/r02_run74_g2.err || exit 1
