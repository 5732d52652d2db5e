# r05 run 8: any-hit candidate lists ordered by hit count (C4); streamed certain reverted; same-box A/B of the round-4
# library (build/ab/libiqpt_r04.so) against this tree: the default line and the share steps with the gather
mkdir -p gpurun_out
O=gpurun_out
R=r05_08
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_bvh.py tests/test_capi.py tests/test_gpu_comm.py tests/test_gpu_certain.py tests/test_gpu_sky.py tests/test_gpu_edge_cases.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -2 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; p=(d.get('per_rank') or [{}])[0]; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), p.get('gather_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'], d['config'].get('kernel_option_bits'))"; }
for ah in 1 0; do
timeout -k 10 400 python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline --anyhit $ah > $O/${R}_c4_ah${ah}.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4_ah${ah}.json c4_anyhit$ah
done
for rep in 1 2; do
for lib in new r04; do
L=""; [ $lib = r04 ] && L="--lib path-tracer-and-rasterizer-engine_amd/build/ab/libiqpt_r04.so"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $L > $O/${R}_n1_${lib}_${rep}.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_n1_${lib}_${rep}.json n1_$lib
for n in 8 4 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather $L > $O/${R}_s${n}g_${lib}_${rep}.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_${lib}_${rep}.json share${n}_$lib
done
done
done
