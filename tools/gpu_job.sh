# r06 run 35: the sky kernel's clamp as a minimum with 1 where |dy| <= 1.5 (bit-identical) against the committed
# library: sky tests, the default line alternated x3
mkdir -p gpurun_out
O=gpurun_out
R=r06_35
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sky.py tests/test_gpu_fullframe.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
for i in 1 2 3; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/${R}_new_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_new_$i.json new$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_head.so > $O/${R}_head_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_head_$i.json head$i
done
