# round-1 GPU run 46: camera-axis formulations A/B with per-round times (alternating order)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab_kernel.py --config c2 --rounds 16 --variants "default=2863,axis=19247,axisS=52015" --out gpurun_out/ab46_c2.json > gpurun_out/ab46_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab46_c2.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/ab46_c2.json'))
for k,v in d['variants'].items(): print(k, v['median_ms'], v['min_ms'], v['bitexact'], v['times_ms'])"
echo DONE
