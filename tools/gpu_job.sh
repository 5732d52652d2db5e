# r03 run 30: XORWOW skip five steps at a time: parity (chain / fan / spec), timelines, shares
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_fan.py tests/test_gpu_chain.py -x -q --timeout 600 --timeout-method thread > $O/r03_30_tests.log 2>&1 || { tail -40 $O/r03_30_tests.log; exit 1; }
tail -1 $O/r03_30_tests.log
for pl in 1 3; do
  timeout -k 10 120 python3 tools/spec_timeline.py --share 8 --specfan 1 --plan $pl --warm 4 --out $O/r03_30_tl_p$pl.json > $O/r03_30_tl_p$pl.log || exit 1
  python3 -c "
import json; d=json.load(open('$O/r03_30_tl_p$pl.json'))
pb = d.get('per_block') or {}
print($pl, d['blocks'], d['kernel_us'], 'slots', d['slots_us']['50'], d['slots_us']['100'], 'iters', d['iters_max_wave']['50'], d['iters_max_wave']['100'], 'walk', d['walk_us']['50'], {k: (v['blocks'], v['slots_us']['50'], v['iters_max_wave']['50'], v['us_per_iter']['50']) for k, v in pb.items() if k.startswith('lanes') and k != 'lanes_hist'})
"
done
for s in 8 4; do
  timeout -k 10 300 python3 bench.py --self-gather --share-of $s --steps 30 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_30_share$s.json 2> $O/r03_30_share$s.err || { tail -20 $O/r03_30_share$s.err; exit 1; }
  tail -1 $O/r03_30_share$s.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['ms_per_step'], d['config']['launch_mode'], d['roofline']['kernel_avg_ms'])"
done
