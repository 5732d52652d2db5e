# round-1 GPU run 58: C5 time split (timing ablations: secondary rays without spheres / without the triangle BVH)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "prim=6951,diag=15143,nosph=15143#8,nobvh=15143#16,neither=15143#24" --out gpurun_out/ab58_c5.json > gpurun_out/ab58_c5.log 2>&1 || { echo FAILED; tail -20 gpurun_out/ab58_c5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab58_c5.json'))
for k,v in d['variants'].items(): print(k, v['median_ms'], v['bitexact'])"
echo DONE
