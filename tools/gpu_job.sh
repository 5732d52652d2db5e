# r04 run 3: spec kernel chains from even start slots with a bounded overshoot (walker falls back to a new
# round at an untraced slot); hybrid N = 1 launches (sphere pixels in the spec kernel beside overlapped plain
# launches): spec / sky / hybrid / certain / multirank tests, C3 shares, N = 1 modes
mkdir -p gpurun_out
O=gpurun_out
R=r04_03
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_hybrid.py tests/test_gpu_sky.py tests/test_gpu_certain.py tests/test_gpu_bench_multirank.py -x -v --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -60 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
line() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['ms_per_step'], d['value'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d.get('gather_check'), d['roofline'].get('kernel_avg_ms'))"; }
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_share$n.json 2> $O/${R}_share$n.err || { tail -20 $O/${R}_share$n.err; exit 1; }
line $O/${R}_share$n.json share$n
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --hybrid on > $O/${R}_hybrid.json 2> $O/${R}_hybrid.err || { tail -20 $O/${R}_hybrid.err; exit 1; }
line $O/${R}_hybrid.json n1_hybrid
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_default.json 2> $O/${R}_default.err || { tail -20 $O/${R}_default.err; exit 1; }
line $O/${R}_default.json n1_default
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --split spec > $O/${R}_n1spec.json 2> $O/${R}_n1spec.err || { tail -20 $O/${R}_n1spec.err; exit 1; }
line $O/${R}_n1spec.json n1_spec
timeout -k 10 120 python3 tools/spec_timeline.py --share 8 > $O/${R}_tl8.log 2>&1 || { tail -20 $O/${R}_tl8.log; exit 1; }
tail -15 $O/${R}_tl8.log
