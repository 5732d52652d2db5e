# r03 run 46: node-test root bounds from v_sqrt_f32 and the NaN fix-ups off the common path: BVH parity, C5 / C4 A/B
# C5 / C4 lines against the previous library (A/B), C5 PMC traffic of the new one
mkdir -p gpurun_out
O=gpurun_out
L=path-tracer-and-rasterizer-engine_amd/iqpt
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_sphere_bvh.py tests/test_gpu_fullframe.py tests/test_gpu_edge_cases.py -x -q --timeout 600 --timeout-method thread > $O/r03_46_tests.log 2>&1 || { tail -40 $O/r03_46_tests.log; exit 1; }
tail -1 $O/r03_46_tests.log
for r in 1 2; do
for v in base new; do
  lib=$L/libiqpt_ab_base.so; [ $v = new ] && lib=$L/libiqpt.so
  timeout -k 10 300 python3 bench.py --lib $lib --config c5 --spp 16 --steps 5 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_46_c5_${v}_$r.json 2> $O/r03_46_c5_${v}_$r.err || { tail -20 $O/r03_46_c5_${v}_$r.err; exit 1; }
  tail -1 $O/r03_46_c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
done
done
for v in base new; do
  lib=$L/libiqpt_ab_base.so; [ $v = new ] && lib=$L/libiqpt.so
  timeout -k 10 300 python3 bench.py --lib $lib --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_46_c4_$v.json 2> $O/r03_46_c4_$v.err || { tail -20 $O/r03_46_c4_$v.err; exit 1; }
  tail -1 $O/r03_46_c4_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
done
P="timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv"
B="python3 bench.py --config c5 --spp 16 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 0"
$P --pmc FETCH_SIZE -d $O/r03_46_c5_fetch -o run -- $B > $O/r03_46_c5_fetch.log 2>&1 || { tail -20 $O/r03_46_c5_fetch.log; exit 1; }
$P --pmc WRITE_SIZE -d $O/r03_46_c5_write -o run -- $B > $O/r03_46_c5_write.log 2>&1 || { tail -20 $O/r03_46_c5_write.log; exit 1; }
python3 tools/pmc_traffic.py $O/r03_46_c5_fetch/run_counter_collection.csv $O/r03_46_c5_write/run_counter_collection.csv c5 $O/r03_46_traffic_c5.json 16 3
python3 -c "import json; d=json.load(open('$O/r03_46_traffic_c5.json')); print('c5 traffic', d['fetch_bytes_corrected'], d['write_bytes'], d['hbm_bytes_per_launch'])"
