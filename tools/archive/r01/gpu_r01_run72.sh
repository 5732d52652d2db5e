# round-1 GPU run 72: C5 BVH-primary at 4 / 5 / 6 waves per SIMD
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "w4=6951,w5=6959,w6=6967" --out gpurun_out/ab72_c5.json > gpurun_out/ab72_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab72_c5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab72_c5.json'))
for k,v in d['variants'].items(): print('c5', k, v['median_ms'], v['bitexact'])"
echo DONE
