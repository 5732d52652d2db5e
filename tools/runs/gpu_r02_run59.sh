# round-2 run 59: rocprofv3 kernel trace + stats of one GPU's C3 N = 2 share through the per-step gather path
# (overlapped launches across the frame copies) and of the default C2 bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_run59_prof_share2 -o share2 --output-format csv -- python3 bench.py --self-gather --share-of 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run59_share2.json 2> gpurun_out/r02_run59_share2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_run59_prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run59_c2.json 2> gpurun_out/r02_run59_c2.err || exit 1
