# r06 run 45: C5 at 16 spp per launch with the 4-wave BVH-primary variant (run 36): the streamed knobs tuned on the
# 5-wave variant in round 5 — per-XCD tile lists above 4 spp (--stream-xcd 1 / 2) and refill groups of 48 — against
# the defaults, alternated x2
mkdir -p gpurun_out
O=gpurun_out
R=r06_45
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('launch_mode'))"; }
for i in 1 2; do
for m in def x1 x2 r48; do
A=""; [ $m = x1 ] && A="--stream-xcd 1"; [ $m = x2 ] && A="--stream-xcd 2"; [ $m = r48 ] && A="--stream-refill 48"
timeout -k 10 200 python3 bench.py --no-cpu-baseline --config c5 --spp 16 --steps 6 --warmup 5 $A > $O/${R}_${m}_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_${m}_$i.json ${m}_$i
done
done
