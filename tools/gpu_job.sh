# r03 run 51: final check of the tree: -m gpu suite, smoke, default bench as the driver runs it (60-s CPU
# baseline), rocprofv3 kernel trace + stats of the default bench
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/r03_51_tests.log 2>&1 || { tail -40 $O/r03_51_tests.log; exit 1; }
tail -1 $O/r03_51_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/r03_51_smoke.log 2>&1 || { tail -20 $O/r03_51_smoke.log; exit 1; }
tail -1 $O/r03_51_smoke.log
timeout -k 10 400 python3 bench.py > $O/r03_51_bench.json 2> $O/r03_51_bench.err || { tail -20 $O/r03_51_bench.err; exit 1; }
tail -1 $O/r03_51_bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03_51_stats -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --verify-rows 0 > $O/r03_51_stats.log 2>&1 || { tail -20 $O/r03_51_stats.log; exit 1; }
tail -1 $O/r03_51_stats.log | cut -c1-300
