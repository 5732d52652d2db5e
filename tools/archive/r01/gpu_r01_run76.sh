# round-1 GPU run 76: C4 BVH-primary work counters (kOptStats), 80-byte vs 64-byte nodes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
for v in node80 new; do
  lib=$L/libiqpt_ab_$v.so; [ $v = new ] && lib=$L/libiqpt_ab.so
  timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c4 --spp 16 --rounds 1 --variants "prim=6959" --stats-opt 6951 --out gpurun_out/ab76_c4_$v.json > gpurun_out/ab76_c4_$v.log 2>&1 || { echo AB4_FAILED $v; tail -20 gpurun_out/ab76_c4_$v.log; exit 1; }
  python3 -c "
import json
d=json.load(open('gpurun_out/ab76_c4_$v.json'))
s=d['stats_default']; print('$v', d['variants']['prim']['median_ms'], s['tri_bvh'], s['sph_bvh'], s['iterations'])"
done
echo DONE
