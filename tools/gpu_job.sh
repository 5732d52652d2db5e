# r06 run 39: the spec kernel at 3 blocks per CU (__launch_bounds__(256, 3): registers without spills; an A/B
# build) against 4 (production): share steps with the gather, alternated x2
mkdir -p gpurun_out
O=gpurun_out
R=r06_39
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for i in 1 2; do
for s in 8 4 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --share-of $s --self-gather > $O/${R}_s${s}_b4_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${s}_b4_$i.json s${s}_b4_$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --share-of $s --self-gather --lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_spec3.so > $O/${R}_s${s}_b3_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${s}_b3_$i.json s${s}_b3_$i
done
done
