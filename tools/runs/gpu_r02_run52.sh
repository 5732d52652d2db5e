# round-2 run 52: chain kernel compile-time knobs (A/B): __launch_bounds__ 4 or 5 waves/SIMD, ring of 1 or 2 slots per
# lane; 16 and 20 chain waves per CU; N = 2, 4, 8 shares
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
for v in libiqpt libiqpt_cw4r1 libiqpt_cw5r1 libiqpt_cw5r2; do
  timeout -k 10 200 python3 tools/split_share.py --lib $L/$v.so --modes chain --ns 2,4,8 --chain-waves 20 --launches 8 --warm 2 > gpurun_out/r02_run52_$v.log 2>&1 || exit 1
done
