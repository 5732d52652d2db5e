# r06 run 26: resident refill group (idle lanes before a plain-kernel wave takes new pixels) 1 (default) / 4 / 16 at
# N = 1 with two rays per lane, alternated x2
mkdir -p gpurun_out
O=gpurun_out
R=r06_26b
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
for i in 1 2 3 4; do
for k in 1 16 64; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --resident-refill $k > $O/${R}_k${k}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_k${k}_$i.json k${k}_$i
done
done
