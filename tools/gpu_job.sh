# r04 run 24: four gather send buffers, frame-buffer ring waits three copies back: tests + share-8 gather parts
mkdir -p gpurun_out
O=gpurun_out
R=r04_24
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['config']['launch_mode'])"; }
for pass in 1 2; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of 8 > $O/${R}_s8_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8_$pass.json s8_nogather
for k in 3 1 2 0; do
timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather --gather-skip $k > $O/${R}_s8_k${k}_$pass.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8_k${k}_$pass.json s8_gather_skip$k
done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_comm.py tests/test_gpu_bench_multirank.py tests/test_gpu_overlap.py tests/test_gpu_hybrid.py tests/test_gpu_facade.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/${R}_prof -o trace -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather > $O/${R}_prof.log 2>&1 || { tail -20 $O/${R}_prof.log; exit 1; }
