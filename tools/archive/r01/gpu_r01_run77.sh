# round-1 GPU run 75 (rerun as 77 with the all-float 64-byte node): 64-byte triangle BVH nodes and packet indices inside the leaf
# pair records: BVH parity tests, then old (previous commit's build, libiqpt_ab_node80.so) vs new C5 / C4
# timing in alternating processes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t77.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t77.log; exit 1; }
tail -2 gpurun_out/t77.log
for pass in 1 2; do
  for v in node80 new; do
    lib=$L/libiqpt_ab_$v.so; [ $v = new ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c5 --spp 1 --rounds 3 --variants "prod=6959" --out gpurun_out/ab77_c5_${v}_$pass.json > gpurun_out/ab77_c5_${v}_$pass.log 2>&1 || { echo AB5_FAILED $v; tail -20 gpurun_out/ab77_c5_${v}_$pass.log; exit 1; }
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c4 --spp 16 --rounds 3 --variants "masks=2855,prim=6959" --out gpurun_out/ab77_c4_${v}_$pass.json > gpurun_out/ab77_c4_${v}_$pass.log 2>&1 || { echo AB4_FAILED $v; tail -20 gpurun_out/ab77_c4_${v}_$pass.log; exit 1; }
    python3 -c "
import json
for c in ('c5','c4'):
    d=json.load(open('gpurun_out/ab77_%s_${v}_$pass.json'%c))
    for k,x in d['variants'].items(): print(c, '$v', $pass, k, x['median_ms'], x['bitexact'])"
  done
done
echo DONE
