# r06 run 50: the committed tree's default line (CPU baseline left out) with run 49's profiles: every profile bench.py
# cites must be of the kernel sources it runs
mkdir -p gpurun_out
O=gpurun_out
R=r06_50
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${R}_default.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_avg_ms'], r['traffic'], r['traffic_same_kernel_sources'], r['mix_same_kernel_sources'], r['executed_work'].get('source'), r['executed_work'].get('missing'))"
