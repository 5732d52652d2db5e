# round-1 GPU run 69: BVH-primary variants without LDS batches / workgroup barriers: GPU suite, C5 and C4 A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t69.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t69.log; exit 1; }
tail -2 gpurun_out/t69.log
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2855,prim=6951" --out gpurun_out/ab69_c5.json > gpurun_out/ab69_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab69_c5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab69_c5.json'))
for k,v in d['variants'].items(): print('c5', k, v['median_ms'], v['bitexact'])"
timeout -k 10 600 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 5 --variants "masks=2855,prim=6951" --out gpurun_out/ab69_c4.json > gpurun_out/ab69_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab69_c4.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab69_c4.json'))
for k,v in d['variants'].items(): print('c4', k, v['median_ms'], v['bitexact'])"
echo DONE
