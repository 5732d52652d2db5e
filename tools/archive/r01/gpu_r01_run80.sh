# round-1 GPU run 80: spheres-first closest hit in production BVH-primary variants: BVH / sphere-BVH parity
# (auto and forced BVH-primary), C5 bench line, C5 stats counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t80.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t80.log; exit 1; }
grep -c PASSED gpurun_out/t80.log
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c5_v2.json --pmc-mix-json profiles/r01_c5_pmc_mix_v1.json > gpurun_out/b80_c5.json 2> gpurun_out/b80_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/b80_c5.err; exit 1; }
cat gpurun_out/b80_c5.json
timeout -k 10 400 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "prim=6959,prim4=6951" --stats-opt 6951 --out gpurun_out/ab80_c5.json > gpurun_out/ab80_c5.log 2>&1 || { echo AB5_FAILED; tail -20 gpurun_out/ab80_c5.log; exit 1; }
python3 -c "
import json
d=json.load(open('gpurun_out/ab80_c5.json'))
for k,x in d['variants'].items(): print('c5', k, x['median_ms'], x['bitexact'])
s=d['stats_default']; print(s['tri_bvh'], s['sph_bvh'])"
echo DONE
