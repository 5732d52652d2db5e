# r03 run 17: the whole -m gpu suite, smoke, then share steps through the gather path and the default bench
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 700 --timeout-method thread > gpurun_out/r03_run17_tests.log 2>&1 || { tail -60 gpurun_out/r03_run17_tests.log; exit 1; }
tail -3 gpurun_out/r03_run17_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_run17_smoke.log 2>&1 || { tail -20 gpurun_out/r03_run17_smoke.log; exit 1; }
tail -1 gpurun_out/r03_run17_smoke.log
for s in 8 4 2; do
  timeout -k 10 180 python -u bench.py --self-gather --share-of $s --no-cpu-baseline --steps 30 > gpurun_out/r03_run17_share$s.json 2> gpurun_out/r03_run17_share$s.err || { tail -20 gpurun_out/r03_run17_share$s.err; exit 1; }
  tail -1 gpurun_out/r03_run17_share$s.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['roofline']['kernel_avg_ms'])"
done
timeout -k 10 300 python -u bench.py --cpu-seconds 10 > gpurun_out/r03_run17_default.json 2> gpurun_out/r03_run17_default.err || { tail -20 gpurun_out/r03_run17_default.err; exit 1; }
tail -1 gpurun_out/r03_run17_default.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'])"
