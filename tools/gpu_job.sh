# r04 run 19: the round-4 tree end to end — pytest -m gpu, smoke, the driver's default bench line, C4 / C5
# lines, share steps with the library gather
mkdir -p gpurun_out
O=gpurun_out
R=r04_19
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), r.get('frac'), r.get('traced_rays_per_s'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'], (d.get('cpu_baseline') or {}).get('value'))"; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/${R}_default.json 2> $O/${R}_default.err || { tail -20 $O/${R}_default.err; exit 1; }
pr $O/${R}_default.json default
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 2 --no-cpu-baseline > $O/${R}_c4.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4.json c4
timeout -k 10 300 python3 bench.py --config c5 --spp 16 --steps 3 --warmup 2 --no-cpu-baseline > $O/${R}_c5.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5.json c5
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather > $O/${R}_s${n}g.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g.json share$n
done
