# r06 run 23: BVH fast accept (a node whose tight box meets [t_min, closest] is visited without the exact test's
# growth) against the same source without it (-DIQPT_BVH_FAST_ACCEPT=0): BVH / sphere-BVH / full-frame tests, C5 lines
mkdir -p gpurun_out
O=gpurun_out
R=r06_23
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py tests/test_gpu_fullframe.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'))"; }
for i in 1 2; do
for v in fa nofa; do
L=""; [ $v = nofa ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_nofa.so"
timeout -k 10 200 python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline $L > $O/${R}_c5_${v}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5_${v}_$i.json c5_16_${v}_$i
timeout -k 10 200 python3 bench.py --config c5 --spp 1 --steps 10 --no-cpu-baseline $L > $O/${R}_c5s1_${v}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s1_${v}_$i.json c5_1_${v}_$i
done
done
