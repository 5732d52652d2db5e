# r05 run 11: queue mode with one-round-trip admissions (per-position records from the prep kernel, cursor
# positions taken ahead) and the walk's chain followed in registers; the spec tests in both modes, timelines
# and share steps
mkdir -p gpurun_out
O=gpurun_out
R=r05_11
export TMPDIR=/tmp
timeout -k 10 240 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 120 --timeout-method thread -k "queue and (launch_sizes or depths or crop)" > $O/${R}_t0.log 2>&1 || { tail -40 $O/${R}_t0.log; exit 1; }
tail -1 $O/${R}_t0.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
for b in 2 3 4; do
for sf in 1 0; do
timeout -k 10 200 python3 tools/spec_timeline.py --share 8 --specfan $sf --queue 1 --qbpc $b --out $O/${R}_tlq_s8_b${b}_sf$sf.json > /dev/null 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/${R}_tlq_s8_b${b}_sf$sf.json')); print('tl b$b sf$sf', d['kernel_us'], d['start_us']['50'], d['end_us'], d['iters']['50'], d['pixels_per_wave']['50'], {k: d[k]['50'] for k in ('admit_us','walk_us','handout_us','trace_us')})"
done
done
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for n in 8 4; do
for b in 3 4 0; do
Q="--spec-queue 1 --spec-qbpc $b"; [ $b = 0 ] && Q="--spec-queue 0"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather $Q > $O/${R}_s${n}g_b$b.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_b$b.json share${n}_b$b
done
done
