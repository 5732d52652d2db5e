# r04 run 21: the share-8 copy path's parts: the render streams' per-launch waits for the frame copies
mkdir -p gpurun_out
O=gpurun_out
R=r04_21
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['config']['launch_mode'])"; }
for pass in 1 2; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of 8 > $O/${R}_s8_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8_$pass.json s8_nogather
for k in 3 7 4; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather --gather-skip $k > $O/${R}_s8_k${k}_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8_k${k}_$pass.json s8_gather_skip$k
done
done
