# r03 run 43: certain-miss (sky) pixels folded at refill: parity, map, default bench, shares
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 120 python3 tools/certain_map.py --out $O/r03_43_certain_map.json | head -1 && timeout -k 10 900 python -u -m pytest tests/test_gpu_certain.py tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_overlap.py tests/test_gpu_edge_cases.py -x -q --timeout 600 --timeout-method thread > $O/r03_43_tests.log 2>&1 || { tail -40 $O/r03_43_tests.log; exit 1; }
tail -1 $O/r03_43_tests.log
for r in 1 2; do
timeout -k 10 300 python3 bench.py --steps 30 --warmup 8 --no-cpu-baseline --verify-rows 8 > $O/r03_43_default_$r.json 2> $O/r03_43_default_$r.err || { tail -20 $O/r03_43_default_$r.err; exit 1; }
tail -1 $O/r03_43_default_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['roofline']['kernel_avg_ms'])"
done
for s in 8 4 2; do
  timeout -k 10 300 python3 bench.py --self-gather --share-of $s --steps 30 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_43_share$s.json 2> $O/r03_43_share$s.err || { tail -20 $O/r03_43_share$s.err; exit 1; }
  tail -1 $O/r03_43_share$s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['ms_per_step'], d['config']['launch_mode'], d['roofline']['kernel_avg_ms'])"
done
