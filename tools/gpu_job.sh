# r03 run 50: certain pixels of streamed scenes folded by iqpt_certain_fold_kernel (the render kernel skips
# them): certain / BVH / full-frame parity, C4 / C5 / C2 lines against run 47's library (A/B)
mkdir -p gpurun_out
O=gpurun_out
L=path-tracer-and-rasterizer-engine_amd/iqpt
timeout -k 10 900 python -u -m pytest tests/test_gpu_certain.py tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py tests/test_gpu_fullframe.py -x -q --timeout 600 --timeout-method thread > $O/r03_50_tests.log 2>&1 || { tail -40 $O/r03_50_tests.log; exit 1; }
tail -1 $O/r03_50_tests.log
for r in 1 2; do
for v in base new; do
  lib=$L/libiqpt_ab_base.so; [ $v = new ] && lib=$L/libiqpt.so
  timeout -k 10 300 python3 bench.py --lib $lib --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_50_c4_${v}_$r.json 2> $O/r03_50_c4_${v}_$r.err || { tail -20 $O/r03_50_c4_${v}_$r.err; exit 1; }
  tail -1 $O/r03_50_c4_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'], d['certain_pixels']['frac_of_rays_counted'])"
  timeout -k 10 300 python3 bench.py --lib $lib --config c5 --spp 16 --steps 5 --warmup 5 --no-cpu-baseline --verify-rows 2 > $O/r03_50_c5_${v}_$r.json 2> $O/r03_50_c5_${v}_$r.err || { tail -20 $O/r03_50_c5_${v}_$r.err; exit 1; }
  tail -1 $O/r03_50_c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'], d['certain_pixels']['frac_of_rays_counted'])"
done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 8 --no-cpu-baseline --verify-rows 4 > $O/r03_50_c2.json 2> $O/r03_50_c2.err || { tail -20 $O/r03_50_c2.err; exit 1; }
tail -1 $O/r03_50_c2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
