# round-2 run 65: rocprofv3 kernel trace + stats of one GPU's C3 N = 2 and N = 8 shares through the gather step
# with bench.py's 8 hardware queues
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_run65_prof_share2 -o share2 --output-format csv -- python3 bench.py --self-gather --share-of 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run65_share2.json 2> gpurun_out/r02_run65_share2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_run65_prof_share8 -o share8 --output-format csv -- python3 bench.py --self-gather --share-of 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run65_share8.json 2> gpurun_out/r02_run65_share8.err || exit 1
