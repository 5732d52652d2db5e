# r03 run 53: the oracle check of the first frame moved after the timed steps; default bench as the
# driver runs it (twice, 5-s CPU baseline) and one GPU's C3 shares N = 8 / 4 / 2, plus the bench-driven
# multi-rank tests
mkdir -p gpurun_out
O=gpurun_out
R=r03_53
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_multirank.py -x -q --timeout 500 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 5 > $O/${R}_default_$k.json 2> $O/${R}_default_$k.err || { tail -20 $O/${R}_default_$k.err; exit 1; }
  tail -1 $O/${R}_default_$k.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['bitexact_frac_vs_oracle'])"
done
for n in 8 4 2; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_share$n.json 2> $O/${R}_share$n.err || { tail -20 $O/${R}_share$n.err; exit 1; }
  tail -1 $O/${R}_share$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share $n', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['gather_check'])"
done
