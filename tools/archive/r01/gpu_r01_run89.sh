# round-1 GPU run 89: BVH-primary at 5 vs 4 waves/SIMD after SAH and spheres-first (C5)
# production 6959 (5 waves, spills) vs 6951 (4 waves, no spills)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 9 --variants "w5=6959,w4=6951" --out gpurun_out/ab89_c5.json > gpurun_out/ab89_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab89_c5.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/ab89_c5.json'))
for k,x in d['variants'].items(): print('c5', k, x['median_ms'], x['bitexact'], x['times_ms'])"
echo DONE
