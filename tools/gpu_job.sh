# r05 run 1: the round-4 A/B options archived (even2, pred, hybrid, specfan); LDS-poison and >64-sphere sky tests;
# pytest -m gpu, smoke, the driver's default line, share steps with the gather
mkdir -p gpurun_out
O=gpurun_out
R=r05_01
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), r.get('frac'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'], (d.get('cpu_baseline') or {}).get('value'))"; }
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather > $O/${R}_s${n}g.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g.json share${n}_gather
done
