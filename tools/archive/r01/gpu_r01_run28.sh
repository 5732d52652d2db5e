# round-1 GPU run 28: full-frame A/B of the camera-ray path (tile masks vs BVH) and of the BVH itself
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2863,prim=6951,-bvh=815" --out gpurun_out/ab28_c5_full.json > gpurun_out/ab28_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab28_c5.log; exit 1; }
head -24 gpurun_out/ab28_c5_full.json
timeout -k 10 400 python tools/ab_kernel.py --config c4 --spp 16 --rounds 3 --variants "masks=2863,prim=6951,-bvh=815" --out gpurun_out/ab28_c4_full.json > gpurun_out/ab28_c4.log 2>&1 || { echo AB4_FAILED; tail -30 gpurun_out/ab28_c4.log; exit 1; }
head -24 gpurun_out/ab28_c4_full.json
echo DONE
