# round-1 GPU run 59: exact sphere BVH: new tests, full GPU suite, C5 A/B and bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sphere_bvh.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/t59a.log 2>&1 || { echo SBVH_TESTS_FAILED; tail -60 gpurun_out/t59a.log; exit 1; }
tail -6 gpurun_out/t59a.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t59.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t59.log; exit 1; }
tail -2 gpurun_out/t59.log
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2855,prim=6951" --out gpurun_out/ab59_c5.json > gpurun_out/ab59_c5.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/ab59_c5.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab59_c5.json'))
for k,v in d['variants'].items(): print(k, v['median_ms'], v['bitexact'])"
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline --steps 5 > gpurun_out/b59_c5.json 2> gpurun_out/b59_c5.err || { echo BENCH5_FAILED; tail -30 gpurun_out/b59_c5.err; exit 1; }
cat gpurun_out/b59_c5.json
echo DONE
