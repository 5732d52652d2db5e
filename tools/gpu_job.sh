# r03 run 25: pipelined spec launches (no per-launch join, async copies on a third stream)
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_bench_multirank.py -x -q --timeout 300 --timeout-method thread > $O/r03_25_tests.log 2>&1 || { tail -40 $O/r03_25_tests.log; exit 1; }
tail -1 $O/r03_25_tests.log
timeout -k 10 600 python3 tools/split_share.py --ns 8,4,2 --modes spec --specfan 1,2 --launches 10 --warm 4 --out $O/r03_25_specfan.json > $O/r03_25_specfan.log 2>&1 || { tail -20 $O/r03_25_specfan.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$O/r03_25_specfan.json'))['rows']:
    print(r['n'], {k: round(v, 4) for k, v in r.items() if k.endswith('ms_median')})
"
for s in 8 4 2; do
  timeout -k 10 300 python3 bench.py --self-gather --share-of $s --split spec --steps 30 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_25_share$s.json 2> $O/r03_25_share$s.err || { tail -20 $O/r03_25_share$s.err; exit 1; }
  tail -1 $O/r03_25_share$s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['ms_per_step'], d['config']['launch_mode'], d['roofline']['kernel_avg_ms'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r03_25_trace_share8 -o run -- python3 bench.py --self-gather --share-of 8 --split spec --steps 20 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_25_trace8.log 2>&1 || { tail -20 $O/r03_25_trace8.log; exit 1; }
