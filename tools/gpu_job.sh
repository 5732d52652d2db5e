# r04 run 34: spec kernel at 5 blocks per CU with the plan's lanes capped at 0.78 of them (= 0.97 of 4 blocks)
mkdir -p gpurun_out
O=gpurun_out
R=r04_34
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for pass in 1 2; do
for cap in 0.78 0.85; do
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of $n --spec-cap $cap > $O/${R}_s${n}_c${cap}_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}_c${cap}_$pass.json share${n}_cap$cap
done
done
done
