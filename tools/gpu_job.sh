# r06 run 20: iqpt_anyhit_kernel batch 4 (default) against A/B builds 2 and 6: C4 lines
mkdir -p gpurun_out
O=gpurun_out
R=r06_20
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for i in 1 2; do
for v in b4 b2 b6; do
L=""; [ $v = b2 ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_any2.so"; [ $v = b6 ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_any6.so"
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline $L > $O/${R}_c4_${v}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4_${v}_$i.json c4_${v}_$i
done
done
