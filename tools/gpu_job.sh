# r04 run 14: timing events bound to the overlapped plain launches' kernels too (N = 1); tests
mkdir -p gpurun_out
O=gpurun_out
R=r04_14
b() { timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@"; }
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d['per_rank'][0] if d.get('per_rank') else {}; print('$2', d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), d['roofline'].get('launch_duration_ms'), p.get('gather_ms'), d.get('gather_check'), d['bitexact_frac_vs_oracle'])"; }
for i in 1 2 3; do
b --steps 20 --warmup 5 > $O/${R}_n1_$i.json 2> $O/${R}_n1_$i.err || { tail -20 $O/${R}_n1_$i.err; exit 1; }
pr $O/${R}_n1_$i.json n1_$i
done
b --steps 20 --warmup 5 --no-kernel-timing > $O/${R}_n1_off.json 2> $O/${R}_n1_off.err || { tail -20 $O/${R}_n1_off.err; exit 1; }
pr $O/${R}_n1_off.json n1_timing_off
b --steps 20 --warmup 5 --share-of 8 --self-gather > $O/${R}_s8g.json 2> $O/${R}_s8g.err || { tail -20 $O/${R}_s8g.err; exit 1; }
pr $O/${R}_s8g.json s8_gather_20steps
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
