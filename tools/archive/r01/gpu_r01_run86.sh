# round-1 GPU run 86: BVH leaf sizes (triangles 2 / 4 / 8 per leaf, spheres 2 / 4 / 8 per leaf; libraries
# built with -DIQPT_LEAF_TRIS / -DIQPT_LEAF_SPHERES) on C5 and the C4 camera-ray BVH, alternating processes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
for pass in 1 2; do
  for v in base t2 t8 s2 s8; do
    lib=$L/libiqpt_ab_$v.so; [ $v = base ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c5 --spp 1 --rounds 3 --variants "prod=6959" --out gpurun_out/ab86_c5_${v}_$pass.json > gpurun_out/ab86_c5_${v}_$pass.log 2>&1 || { echo AB5_FAILED $v; tail -20 gpurun_out/ab86_c5_${v}_$pass.log; exit 1; }
    python3 -c "
import json
d=json.load(open('gpurun_out/ab86_c5_${v}_$pass.json'))
for k,x in d['variants'].items(): print('c5', '$v', $pass, k, x['median_ms'], x['times_ms'])"
  done
  for v in base t2 t8; do
    lib=$L/libiqpt_ab_$v.so; [ $v = base ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c4 --spp 16 --rounds 3 --variants "masks=2855,prim=6959" --out gpurun_out/ab86_c4_${v}_$pass.json > gpurun_out/ab86_c4_${v}_$pass.log 2>&1 || { echo AB4_FAILED $v; tail -20 gpurun_out/ab86_c4_${v}_$pass.log; exit 1; }
    python3 -c "
import json
d=json.load(open('gpurun_out/ab86_c4_${v}_$pass.json'))
for k,x in d['variants'].items(): print('c4', '$v', $pass, k, x['median_ms'])"
  done
done
echo DONE
