# r06 run 17: BVH successor touches (-DIQPT_BVH_PREFETCH=1) against the default build, C5 at 16 and 1 spp, alternated
mkdir -p gpurun_out
O=gpurun_out
R=r06_17
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'))"; }
for i in 1 2; do
for v in base pf1; do
L=""; [ $v = pf1 ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_pf1.so"
timeout -k 10 200 python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline $L > $O/${R}_c5_${v}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5_${v}_$i.json c5_16_${v}_$i
timeout -k 10 200 python3 bench.py --config c5 --spp 1 --steps 10 --no-cpu-baseline $L > $O/${R}_c5s1_${v}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s1_${v}_$i.json c5_1_${v}_$i
done
done
