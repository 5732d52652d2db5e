# r05 run 40: per-XCD queues for streamed launches of up to 4 spp (iqpt_debug_set_stream_xcd 3, the default):
# BVH / full-frame / overlap tests, smoke, the C5 line at 1 / 4 / 16 spp and C4 against one queue (mode 0),
# the default line, rocprofv3 kernel stats of the C5 16-spp line
mkdir -p gpurun_out
O=gpurun_out
R=r05_40
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_fullframe.py tests/test_gpu_overlap.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], r.get('frac'), c.get('value'))"; }
for s in 1 4 16; do
st=10; [ $s = 1 ] && st=40; [ $s = 4 ] && st=20
for m in 3 0; do
timeout -k 10 240 python3 bench.py --config c5 --spp $s --steps $st --no-cpu-baseline --stream-xcd $m > $O/${R}_c5s${s}_x$m.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s${s}_x$m.json c5_${s}spp_x$m
done
done
timeout -k 10 240 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > $O/${R}_c4.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4.json c4
timeout -k 10 300 python3 bench.py > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_c5 -o run -- python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline > $O/${R}_prof_c5.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_c5.json prof_c5
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_c5s1 -o run -- python3 bench.py --config c5 --steps 40 --no-cpu-baseline > $O/${R}_prof_c5s1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_c5s1.json prof_c5_default
