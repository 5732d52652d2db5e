# r03 run 49: the tree after the C5 register diet: default bench (CPU baseline), C3 share steps N = 8 / 4 / 2
# through the gather path, C4 / C5 lines
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python3 bench.py --cpu-seconds 20 > $O/r03_49_default.json 2> $O/r03_49_default.err || { tail -20 $O/r03_49_default.err; exit 1; }
tail -1 $O/r03_49_default.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('default', d['value'], d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['roofline']['kernel_avg_ms'], d['cpu_baseline']['value'])"
for r in 1 2; do
for s in 8 4 2; do
  timeout -k 10 300 python3 bench.py --self-gather --share-of $s --steps 30 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_49_share${s}_$r.json 2> $O/r03_49_share${s}_$r.err || { tail -20 $O/r03_49_share${s}_$r.err; exit 1; }
  tail -1 $O/r03_49_share${s}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share', $s, d['ms_per_step'], d['config']['launch_mode'], d['roofline']['kernel_avg_ms'], d.get('gather_check'))"
done
done
timeout -k 10 300 python3 bench.py --config c5 --spp 16 --steps 5 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_49_c5.json 2> $O/r03_49_c5.err || { tail -20 $O/r03_49_c5.err; exit 1; }
tail -1 $O/r03_49_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'], d['roofline']['hbm'])"
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_49_c4.json 2> $O/r03_49_c4.err || { tail -20 $O/r03_49_c4.err; exit 1; }
tail -1 $O/r03_49_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
