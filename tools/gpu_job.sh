# r03 run 57: final check of the tree: -m gpu suite, smoke, default bench as the driver runs it (5-s CPU
# baseline), rocprofv3 kernel trace + stats of the default bench
mkdir -p gpurun_out
O=gpurun_out
R=r03_57
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 5 > $O/${R}_bench.json 2> $O/${R}_bench.err || { tail -20 $O/${R}_bench.err; exit 1; }
tail -1 $O/${R}_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_stats -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_stats.log 2>&1 || { tail -20 $O/${R}_stats.log; exit 1; }
grep '^{' $O/${R}_stats.log | cut -c1-200
