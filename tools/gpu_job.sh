# r06 run 15: two-ray pair test with T = O - v0 held ahead of the determinant test (one LDS wait per pair) against
# the same source without it (-DIQPT_PAIR2_PIN=0), alternated, the default line; pipe tests
mkdir -p gpurun_out
O=gpurun_out
R=r06_15
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_fullframe.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'))"; }
for i in 1 2 3; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/${R}_pin_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_pin_$i.json pin$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_nopin.so > $O/${R}_nopin_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_nopin_$i.json nopin$i
done
