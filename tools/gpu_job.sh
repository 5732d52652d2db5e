# r06 run 46: overlapped N = 1 launches with fewer blocks per CU each (A/B builds -DIQPT_OVL_OCC_DEC=2 / 3: occupancy
# less 2 / 3 instead of less 1), C2 default line (K = 100), alternated x3
mkdir -p gpurun_out
O=gpurun_out
R=r06_46
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for i in 1 2 3; do
for m in def d2 d3; do
A=""; [ $m = d2 ] && A="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_occdec2.so"; [ $m = d3 ] && A="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_occdec3.so"
timeout -k 10 200 python3 bench.py --no-cpu-baseline $A > $O/${R}_${m}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_${m}_$i.json ${m}_$i
done
done
