# round-1 GPU run 66: C4 candidate-list loop, software-pipelined pair loads (kOptExp) vs plain
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 7 --variants "masks=2855,pipe=35623" --out gpurun_out/ab66_c4.json > gpurun_out/ab66_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab66_c4.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab66_c4.json'))
for k,v in d['variants'].items(): print('c4', k, v['median_ms'], v['bitexact'])"
echo DONE
