# r06 run 25b: spec window margins 1/16 (default), 1/32, 1/1000 at the share-8 / share-4 steps
mkdir -p gpurun_out
O=gpurun_out
R=r06_25b
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for s in 8 4; do
for m in 16 32 1000 16; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --share-of $s --spec-margin $m > $O/${R}_s${s}_m$m.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${s}_m$m.json s${s}_m$m
done
done
