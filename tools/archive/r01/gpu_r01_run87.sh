# round-1 GPU run 87: triangle leaves of 8 vs 4 (repeat of run 86 with more passes)
# (libiqpt_ab_t8.so built with -DIQPT_LEAF_TRIS=8), C5 and the C4 camera-ray BVH
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
for pass in 1 2 3; do
  for v in base t8; do
    lib=$L/libiqpt_ab_$v.so; [ $v = base ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c5 --spp 1 --rounds 3 --variants "prod=6959" --out gpurun_out/ab87_c5_${v}_$pass.json > gpurun_out/ab87_c5_${v}_$pass.log 2>&1 || { echo AB5_FAILED $v; tail -20 gpurun_out/ab87_c5_${v}_$pass.log; exit 1; }
    python3 -c "
import json
d=json.load(open('gpurun_out/ab87_c5_${v}_$pass.json'))
for k,x in d['variants'].items(): print('c5', '$v', $pass, k, x['median_ms'], x['times_ms'])"
  done
  for v in base t8; do
    lib=$L/libiqpt_ab_$v.so; [ $v = base ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c4 --spp 16 --rounds 3 --variants "masks=2855,prim=6959" --out gpurun_out/ab87_c4_${v}_$pass.json > gpurun_out/ab87_c4_${v}_$pass.log 2>&1 || { echo AB4_FAILED $v; tail -20 gpurun_out/ab87_c4_${v}_$pass.log; exit 1; }
    python3 -c "
import json
d=json.load(open('gpurun_out/ab87_c4_${v}_$pass.json'))
for k,x in d['variants'].items(): print('c4', '$v', $pass, k, x['median_ms'])"
  done
done
echo DONE
