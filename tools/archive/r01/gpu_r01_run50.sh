# round-1 GPU run 50: launch-tail check: kernel time vs spp per launch, default vs camera-axis variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r50.txt
for spp in 16 64 256; do
for v in 2863 19247; do
timeout -k 10 120 python3 tools/ab_kernel.py --config c2 --spp $spp --only $v --frames 10 | sed "s/^/spp=$spp /" >> gpurun_out/r50.txt 2> gpurun_out/r50.err || { echo FAILED $v; tail -20 gpurun_out/r50.err; exit 1; }
done
done
cat gpurun_out/r50.txt
echo DONE
