# r03 run 47: 0.5 z of the scalar cosine polynomial as v_ldexp_f32 (no packed constant pair to spill): full
# -m gpu suite, C5 / C4 / C2 lines against the run-46 library (A/B), C5 PMC traffic of the new one
mkdir -p gpurun_out
O=gpurun_out
L=path-tracer-and-rasterizer-engine_amd/iqpt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/r03_47_tests.log 2>&1 || { tail -40 $O/r03_47_tests.log; exit 1; }
tail -1 $O/r03_47_tests.log
for r in 1 2; do
for v in base new; do
  lib=$L/libiqpt_ab_base.so; [ $v = new ] && lib=$L/libiqpt.so
  timeout -k 10 300 python3 bench.py --lib $lib --config c5 --spp 16 --steps 5 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_47_c5_${v}_$r.json 2> $O/r03_47_c5_${v}_$r.err || { tail -20 $O/r03_47_c5_${v}_$r.err; exit 1; }
  tail -1 $O/r03_47_c5_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
  timeout -k 10 300 python3 bench.py --lib $lib --steps 20 --warmup 8 --no-cpu-baseline --verify-rows 4 > $O/r03_47_c2_${v}_$r.json 2> $O/r03_47_c2_${v}_$r.err || { tail -20 $O/r03_47_c2_${v}_$r.err; exit 1; }
  tail -1 $O/r03_47_c2_${v}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'], d['certain_pixels']['frac_of_rays_counted'])"
done
done
for v in base new; do
  lib=$L/libiqpt_ab_base.so; [ $v = new ] && lib=$L/libiqpt.so
  timeout -k 10 300 python3 bench.py --lib $lib --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_47_c4_$v.json 2> $O/r03_47_c4_$v.err || { tail -20 $O/r03_47_c4_$v.err; exit 1; }
  tail -1 $O/r03_47_c4_$v.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', '$v', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
done
P="timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv"
B="python3 bench.py --config c5 --spp 16 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 0"
$P --pmc FETCH_SIZE -d $O/r03_47_c5_fetch -o run -- $B > $O/r03_47_c5_fetch.log 2>&1 || { tail -20 $O/r03_47_c5_fetch.log; exit 1; }
$P --pmc WRITE_SIZE -d $O/r03_47_c5_write -o run -- $B > $O/r03_47_c5_write.log 2>&1 || { tail -20 $O/r03_47_c5_write.log; exit 1; }
python3 tools/pmc_traffic.py $O/r03_47_c5_fetch/run_counter_collection.csv $O/r03_47_c5_write/run_counter_collection.csv c5 $O/r03_47_traffic_c5.json 16 3
python3 -c "import json; d=json.load(open('$O/r03_47_traffic_c5.json')); print('c5 traffic', d['fetch_bytes_corrected'], d['write_bytes'], d['hbm_bytes_per_launch'])"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 -d $O/r03_47_mixa -o run -- $B > $O/r03_47_mixa.log 2>&1 || { tail -20 $O/r03_47_mixa.log; exit 1; }
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/r03_47_mixb -o run -- $B > $O/r03_47_mixb.log 2>&1 || { tail -20 $O/r03_47_mixb.log; exit 1; }
python3 tools/pmc_mix.py $O/r03_47_mixa/run_counter_collection.csv $O/r03_47_mixb/run_counter_collection.csv c5 1 $O/r03_c5_pmc_mix_v4.json "iqpt_render_kernel C5 16 spp (last dispatch; per_iteration = per launch)" > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/r03_c5_pmc_mix_v4.json')); print('c5 mix', d['counters']['SQ_INSTS_VALU'], d['kernel_ms_profiled'], d['valu_busy_frac'], d['wave_time_split'], d['mean_waves_per_simd'])"
