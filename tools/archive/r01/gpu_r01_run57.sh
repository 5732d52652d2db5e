# round-1 GPU run 57: 6 waves/SIMD variants (with / without the camera-axis transform), 20-frame averages
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r57.txt
for r in 1 2; do
for v in 2863 2879 19255; do
timeout -k 10 120 python3 tools/ab_kernel.py --config c2 --only $v --frames 20 >> gpurun_out/r57.txt 2> gpurun_out/r57.err || { echo FAILED $v; tail -20 gpurun_out/r57.err; exit 1; }
done
done
cat gpurun_out/r57.txt
echo DONE
