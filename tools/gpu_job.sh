# r04 run 25: predicted chains in the spec kernel (camera rays of every slot, scattered rays along the chain as
# predicted): the new tests, the spec tests, shares with it on and off, N = 1 spec
mkdir -p gpurun_out
O=gpurun_out
R=r04_25
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec_pred.py -x -v --timeout 120 --timeout-method thread > $O/${R}_tests_pred.log 2>&1 || { tail -40 $O/${R}_tests_pred.log; exit 1; }
tail -2 $O/${R}_tests_pred.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_spec_even.py tests/test_gpu_hybrid.py tests/test_gpu_bench_multirank.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for pr_ in on off; do
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of $n --spec-pred $pr_ > $O/${R}_s${n}_$pr_.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}_$pr_.json share${n}_nogather_pred_$pr_
done
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather --spec-pred $pr_ > $O/${R}_s8g_$pr_.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8g_$pr_.json share8_gather_pred_$pr_
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --split spec --spec-pred $pr_ > $O/${R}_n1spec_$pr_.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1spec_$pr_.json n1_spec_pred_$pr_
done
