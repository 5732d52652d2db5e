# r04 run 8: host time per step inside iqpt_render / iqpt_gather_frame_async (share 8, self-gather) and N = 1
mkdir -p gpurun_out
O=gpurun_out
R=r04_08
b() { timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline "$@"; }
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), d.get('per_rank'))"; }
b --share-of 8 --self-gather > $O/${R}_s8g.json 2> $O/${R}_s8g.err || { tail -20 $O/${R}_s8g.err; exit 1; }
pr $O/${R}_s8g.json s8_gather
b --share-of 8 --self-gather --sky off > $O/${R}_s8g_skyoff.json 2> $O/${R}_s8g_skyoff.err || { tail -20 $O/${R}_s8g_skyoff.err; exit 1; }
pr $O/${R}_s8g_skyoff.json s8_gather_skyoff
b --share-of 4 --self-gather > $O/${R}_s4g.json 2> $O/${R}_s4g.err || { tail -20 $O/${R}_s4g.err; exit 1; }
pr $O/${R}_s4g.json s4_gather
