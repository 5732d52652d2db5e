# round-1 GPU run 83: miss successor node loaded during the node test (kOptExp) vs production,
# C5 and C4 (BVH-primary at 5 and 4 waves)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 7 --variants "prod=6959,pre=39727,prod4=6951,pre4=39719" --out gpurun_out/ab83_c5.json > gpurun_out/ab83_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab83_c5.log; exit 1; }
timeout -k 10 400 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 5 --variants "prim=6959,pre=39727" --out gpurun_out/ab83_c4.json > gpurun_out/ab83_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab83_c4.log; exit 1; }
python3 -c "
import json
for c in ('c5','c4'):
    d=json.load(open('gpurun_out/ab83_%s.json'%c))
    for k,x in d['variants'].items(): print(c, k, x['median_ms'], x['bitexact'], x['times_ms'])"
echo DONE
