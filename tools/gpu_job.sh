# r04 run 28: spec lane classes 24 and 48 besides 8, 16, 32, 64 (a plan can use the 5th resident block): tests, shares
mkdir -p gpurun_out
O=gpurun_out
R=r04_28
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_spec_pred.py tests/test_gpu_spec_even.py tests/test_gpu_bench_multirank.py tests/test_gpu_hybrid.py tests/test_gpu_comm.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'])"; }
for pass in 1 2; do
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of $n > $O/${R}_s${n}_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}_$pass.json share${n}_nogather
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of $n --self-gather > $O/${R}_s${n}g_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_$pass.json share${n}_gather
done
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${R}_prof -o trace -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --share-of 8 > $O/${R}_prof.log 2>&1 || { tail -20 $O/${R}_prof.log; exit 1; }
