# r05 run 27: resident any-hit form (spheres first, then triangles until one is accepted closer; kOptAnyHit
# variants chosen by launch_render / launch_spec for scenes under the reference's materials): parity tests, then
# the default line and share steps against the previous library (build/ab/libiqpt_r05b.so), alternated
mkdir -p gpurun_out
O=gpurun_out
R=r05_27
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py tests/test_gpu_overlap.py tests/test_gpu_sky.py tests/test_gpu_certain.py tests/test_gpu_edge_cases.py tests/test_golden.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 200 --timeout-method thread -k block > $O/${R}_tests2.log 2>&1 || { tail -40 $O/${R}_tests2.log; exit 1; }
tail -1 $O/${R}_tests2.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'))"; }
for rep in 1 2; do
for lib in new old; do
L=""; [ $lib = old ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/ab/libiqpt_r05b.so"
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $L > $O/${R}_n1_${lib}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1_${lib}_$rep.json n1_$lib
for n in 8 2; do
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather $L > $O/${R}_s${n}g_${lib}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_${lib}_$rep.json share${n}_$lib
done
done
done
