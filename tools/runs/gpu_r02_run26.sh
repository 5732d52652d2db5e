# round-2 run 26: packed branch-free scatter transcendentals (kOptScatter2): libm bit-identity, C2 A/B,
# lone-wave sphere-tile latency
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_libm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_run26_libm.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_kernel.py --config c2 --rounds 11 --variants prio=133935,scatter2=396079,noprio=2863 --stats-opt 396079 --out gpurun_out/r02_ab_scatter2.json > gpurun_out/r02_run26_ab.log 2>&1 || exit 1
LONE_OPT=133935 timeout -k 10 200 python -u tools/lone_wave.py gpurun_out/r02_lone_prio.json > gpurun_out/r02_run26_lone.log 2>&1 || exit 1
LONE_OPT=396079 timeout -k 10 200 python -u tools/lone_wave.py gpurun_out/r02_lone_scatter2.json >> gpurun_out/r02_run26_lone.log 2>&1 || exit 1
