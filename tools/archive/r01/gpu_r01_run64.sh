# round-1 GPU run 64: C4 time split: with / without the pair tests (batch streaming only)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 5 --variants "masks=2855,diag=11047,notest=11047#32" --out gpurun_out/ab64_c4.json > gpurun_out/ab64_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab64_c4.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab64_c4.json'))
for k,v in d['variants'].items(): print('c4', k, v['median_ms'], v['bitexact'])"
echo DONE
