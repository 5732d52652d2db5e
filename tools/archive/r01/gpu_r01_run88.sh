# round-1 GPU run 88: BVH-primary closest hit ordered always-list spheres -> triangles -> sphere BVH
# (kOptExp, 39727) against spheres -> triangles (production 6959): C5 timing + bit-exactness
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 9 --variants "prod=6959,ground=39727" --out gpurun_out/ab88_c5.json > gpurun_out/ab88_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab88_c5.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/ab88_c5.json'))
for k,x in d['variants'].items(): print('c5', k, x['median_ms'], x['bitexact'], x['times_ms'])"
echo DONE
