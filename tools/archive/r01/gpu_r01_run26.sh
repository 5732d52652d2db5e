# round-1 GPU run 26: block-level skip of the triangle batches; A/B camera rays through the BVH (C5 crop)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t26.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t26.log; exit 1; }
tail -2 gpurun_out/t26.log
timeout -k 10 300 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --crop 0,3840,0,54,40 --variants "default=2863,prim=6951,-bvh=815" --out gpurun_out/ab26_c5_prim.json > gpurun_out/ab26_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab26_c5.log; exit 1; }
head -30 gpurun_out/ab26_c5_prim.json
timeout -k 10 300 python tools/ab_kernel.py --config c4 --spp 4 --rounds 3 --crop 0,1920,0,27,40 --variants "default=2863,prim=6951" --out gpurun_out/ab26_c4_prim.json > gpurun_out/ab26_c4.log 2>&1 || { echo AB4_FAILED; tail -30 gpurun_out/ab26_c4.log; exit 1; }
head -20 gpurun_out/ab26_c4_prim.json
echo DONE
