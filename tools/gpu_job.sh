# r05 run 13: queue mode with the walk's chain from jump tables (6 lookups per lane instead of 64 dependent
# steps), checkpoints every 8 slots, fewer lane registers; spec tests, timeline, share steps
mkdir -p gpurun_out
O=gpurun_out
R=r05_13
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
for b in 3 4; do
timeout -k 10 200 python3 tools/spec_timeline.py --share 8 --specfan 1 --queue 1 --qbpc $b --out $O/${R}_tlq_s8_b${b}_sf1.json > /dev/null 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${R}_tlq_s8_b${b}_sf1.json')); print('tl b$b sf1', d['kernel_us'], d['end_us'], {k: d[k]['50'] for k in d if k.endswith('_us') and isinstance(d[k], dict) and '50' in d[k]})"
done
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for rep in 1 2; do
for n in 8 4; do
for b in 4 0; do
Q="--spec-queue 1 --spec-qbpc $b"; [ $b = 0 ] && Q="--spec-queue 0"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather $Q > $O/${R}_s${n}g_b${b}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_b${b}_$rep.json share${n}_b$b
done
done
done
