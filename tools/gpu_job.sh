# r05 run 22: the bench lines with the committed round-5 profiles (executed work keyed on these kernel sources,
# PMC traffic / mixes of r05): the default line, C4, C5, the share-8 step
mkdir -p gpurun_out
O=gpurun_out
R=r05_22
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), r.get('frac'), (r.get('executed_work') or {}).get('frac'), (r.get('executed_work') or {}).get('source') or (r.get('executed_work') or {}).get('missing'), r.get('mix_source'), (r.get('hbm') or {}).get('pmc_source'), d['bitexact_frac_vs_oracle'])"; }
timeout -k 10 170 python3 bench.py > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
timeout -k 10 170 python3 bench.py --config c5 --spp 16 --steps 8 --warmup 5 --no-cpu-baseline > $O/${R}_c5.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5.json c5
timeout -k 10 170 python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline > $O/${R}_c4.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4.json c4
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather > $O/${R}_s8g.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8g.json share8
