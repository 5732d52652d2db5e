# r03 run 56: spec plan lane cap A/B through bench.py's share steps (--self-gather, 8 hardware queues,
# stream-ordered copies), N = 4 and 8, caps interleaved over two rounds
mkdir -p gpurun_out
O=gpurun_out
R=r03_56
for r in 1 2; do
  for n in 4 8; do
    for cap in 0.97 0.75 1.1; do
      timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline --spec-cap $cap > $O/${R}_s${n}_c${cap}_$r.json 2> $O/${R}_s${n}_c${cap}_$r.err || { tail -20 $O/${R}_s${n}_c${cap}_$r.err; exit 1; }
      tail -1 $O/${R}_s${n}_c${cap}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('share $n cap $cap', d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['bitexact_frac_vs_oracle'], d['gather_check'])"
    done
  done
done
