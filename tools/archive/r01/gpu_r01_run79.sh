# round-1 GPU run 79: spheres before triangles on the BVH-primary path (kOptExp A/B, 39727) against the
# production order (6959; both with the always-tested spheres first in the sphere pass); sphere/BVH parity
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t79.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t79.log; exit 1; }
tail -2 gpurun_out/t79.log
timeout -k 10 400 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 7 --variants "prod=6959,sfirst=39727" --out gpurun_out/ab79_c5.json > gpurun_out/ab79_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab79_c5.log; exit 1; }
timeout -k 10 400 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 5 --variants "masks=2855,prim=6959,sfirst=39727" --out gpurun_out/ab79_c4.json > gpurun_out/ab79_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab79_c4.log; exit 1; }
python3 -c "
import json
for c in ('c5','c4'):
    d=json.load(open('gpurun_out/ab79_%s.json'%c))
    for k,x in d['variants'].items(): print(c, k, x['median_ms'], x['bitexact'], x['times_ms'])"
echo DONE
