# r04 run 17: even slots of 2-slot sphere pixels as an option (kspec::even2): tests, the 8-rank one-GPU
# rehearsal with it on and off, share steps and N = 1 spec / hybrid with it on and off
mkdir -p gpurun_out
O=gpurun_out
R=r04_17
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec_even.py tests/test_gpu_spec.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
for ev in on off; do
timeout -k 10 300 python3 bench.py --gpus 8 --steps 2 --warmup 1 --no-cpu-baseline --verify-rows 2 --backend gloo --one-device --spec-even $ev > $O/${R}_n8_$ev.json 2> $O/${R}_n8_$ev.err || { tail -30 $O/${R}_n8_$ev.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${R}_n8_$ev.json').read().strip().splitlines()[-1]); print('n8_rehearsal_even_$ev', d['bitexact_frac_vs_oracle'], d['config']['launch_mode'], [(p['rank'], p['bitexact_frac_vs_oracle']) for p in d['per_rank']])"
done
b() { timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 40 --warmup 5 "$@"; }
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); p=d['per_rank'][0] if d.get('per_rank') else {}; print('$2', d['ms_per_step'], d['roofline'].get('kernel_avg_ms'), p.get('gather_ms'), d.get('gather_check'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for ev in on off; do
for n in 8 4 2; do
b --share-of $n --self-gather --spec-even $ev > $O/${R}_s${n}g_$ev.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_$ev.json s${n}_gather_even_$ev
done
b --share-of 8 --spec-even $ev > $O/${R}_s8_$ev.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8_$ev.json s8_nogather_even_$ev
b --split spec --spec-even $ev > $O/${R}_n1spec_$ev.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1spec_$ev.json n1_spec_even_$ev
b --hybrid on --spec-even $ev > $O/${R}_n1hyb_$ev.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1hyb_$ev.json n1_hybrid_even_$ev
done
b > $O/${R}_n1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1.json n1_default
