# r06 run 27: the final tree's C3 share steps with the library's gather (N = 8 / 4 / 2, x2), C5 at 1 spp per step
mkdir -p gpurun_out
O=gpurun_out
R=r06_27
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for i in 1 2; do
for s in 8 4 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --share-of $s --self-gather > $O/${R}_s${s}g_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${s}g_$i.json s${s}g_$i
done
done
timeout -k 10 200 python3 bench.py --config c5 --spp 1 --steps 10 --no-cpu-baseline > $O/${R}_c5s1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s1.json c5_spp1
