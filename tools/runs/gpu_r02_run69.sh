# round-2 run 69: rocprofv3 kernel trace of one GPU's C3 N = 8 share through the gather step after the chain
# stream-order change
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_run69_prof_share8 -o share8 --output-format csv -- python3 bench.py --self-gather --share-of 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run69_share8.json 2> gpurun_out/r02_run69_share8.err || exit 1
