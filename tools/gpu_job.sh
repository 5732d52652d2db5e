# r04 run 2: sky kernel for certain-miss pixels (test_gpu_sky); libiqpt's RCCL gather (iqpt_comm_*), facade sharded path, multirank bench tests; spec kernel as
# coalescing chains (parity: test_gpu_spec / fan / certain); default bench and C3 shares
mkdir -p gpurun_out
O=gpurun_out
R=r04_02
timeout -k 10 900 python -u -m pytest tests/test_gpu_sky.py tests/test_gpu_spec.py tests/test_gpu_comm.py tests/test_gpu_facade.py tests/test_gpu_bench_multirank.py -x -v --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -60 $O/${R}_tests.log; exit 1; }
tail -3 $O/${R}_tests.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 5 > $O/${R}_bench.json 2> $O/${R}_bench.err || { tail -20 $O/${R}_bench.err; exit 1; }
tail -1 $O/${R}_bench.json | cut -c1-300
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --self-gather --share-of $n --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_share$n.json 2> $O/${R}_share$n.err || { tail -20 $O/${R}_share$n.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$O/${R}_share$n.json').read().strip().splitlines()[-1]); print('share$n', d['ms_per_step'], d['config']['launch_mode'], d['bitexact_frac_vs_oracle'], d['gather_check'], d['per_rank'])"
done
