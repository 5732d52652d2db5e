# r05 run 34: refill group size for streamed scenes beyond 16: C5 16 spp per launch K = 16 / 32 / 48 / 64 x2 and C5
# at 1 spp per launch (the progressive pass) K = 1 / 16 / 32 / 64 x2, alternated
mkdir -p gpurun_out
O=gpurun_out
R=r05_34
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
for rep in 1 2; do
for k in 16 32 48 64; do
timeout -k 10 240 python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline --stream-refill $k > $O/${R}_c5_k${k}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5_k${k}_$rep.json c5_16spp_k${k}_$rep
done
for k in 1 16 32 64; do
timeout -k 10 240 python3 bench.py --config c5 --spp 1 --steps 40 --no-cpu-baseline --stream-refill $k > $O/${R}_c5s1_k${k}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s1_k${k}_$rep.json c5_1spp_k${k}_$rep
done
done
