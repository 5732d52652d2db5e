# r05 run 26: the N = 1 line under each launch mode (sphere tiles in a dispatch of their own —
# FAN: split tiles in the plain kernel beside the fan kernel; CHAIN; SPEC; auto = overlapped plain launches)
mkdir -p gpurun_out
O=gpurun_out
R=r05_26
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for rep in 1 2; do
for m in auto fan chain spec; do
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --split $m > $O/${R}_n1_$m_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1_$m_$rep.json n1_$m
done
done
