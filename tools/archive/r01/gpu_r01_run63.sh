# round-1 GPU run 63: uniform-tile mask words on the streamed path: GPU suite, C4/C5 A/B, bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t63.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t63.log; exit 1; }
tail -2 gpurun_out/t63.log
timeout -k 10 600 python3 tools/ab_kernel.py --config c4 --spp 16 --rounds 5 --variants "masks=2855,prim=6951" --out gpurun_out/ab63_c4.json > gpurun_out/ab63_c4.log 2>&1 || { echo AB4_FAILED; tail -20 gpurun_out/ab63_c4.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab63_c4.json'))
for k,v in d['variants'].items(): print('c4', k, v['median_ms'], v['bitexact'])"
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2855,prim=6951" --out gpurun_out/ab63_c5.json > gpurun_out/ab63_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab63_c5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab63_c5.json'))
for k,v in d['variants'].items(): print('c5', k, v['median_ms'], v['bitexact'])"
timeout -k 10 400 python bench.py --config c4 --spp 16 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/b63_c4.json 2> gpurun_out/b63_c4.err || { echo BENCH4_FAILED; tail -30 gpurun_out/b63_c4.err; exit 1; }
cat gpurun_out/b63_c4.json
echo DONE
