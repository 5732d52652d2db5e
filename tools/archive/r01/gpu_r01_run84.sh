# round-1 GPU run 84: binned-SAH BVH builds (triangles and spheres) against the median-split builds
# (libiqpt_ab_median.so = previous commit): BVH parity tests, then C5 / C4 timing in alternating processes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t84.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t84.log; exit 1; }
tail -1 gpurun_out/t84.log
for pass in 1 2; do
  for v in median sah; do
    lib=$L/libiqpt_ab_$v.so; [ $v = sah ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c5 --spp 1 --rounds 3 --variants "prod=6959" --stats-opt 6951 --out gpurun_out/ab84_c5_${v}_$pass.json > gpurun_out/ab84_c5_${v}_$pass.log 2>&1 || { echo AB5_FAILED $v; tail -20 gpurun_out/ab84_c5_${v}_$pass.log; exit 1; }
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c4 --spp 16 --rounds 3 --variants "masks=2855,prim=6959" --out gpurun_out/ab84_c4_${v}_$pass.json > gpurun_out/ab84_c4_${v}_$pass.log 2>&1 || { echo AB4_FAILED $v; tail -20 gpurun_out/ab84_c4_${v}_$pass.log; exit 1; }
    python3 -c "
import json
for c in ('c5','c4'):
    d=json.load(open('gpurun_out/ab84_%s_${v}_$pass.json'%c))
    for k,x in d['variants'].items(): print(c, '$v', $pass, k, x['median_ms'], x['bitexact'])
    s=d.get('stats_default')
    if c=='c5' and s: print('   tri', s['tri_bvh'], 'sph', s['sph_bvh'])"
  done
done
echo DONE
