# round-1 GPU run 48: kernel time per variant, 20-frame averages, alternating processes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r48.txt
for r in 1 2 3; do
for v in 2863 19247 52015; do
timeout -k 10 120 python3 tools/ab_kernel.py --config c2 --only $v --frames 20 >> gpurun_out/r48.txt 2> gpurun_out/r48.err || { echo FAILED $v; tail -20 gpurun_out/r48.err; exit 1; }
done
done
cat gpurun_out/r48.txt
echo DONE
