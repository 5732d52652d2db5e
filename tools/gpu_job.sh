# r03 run 42: certain pixels for resident scenes only: C4 / C5 back, C2 default, kernel-trace stats and the
# instruction mix of the C2 kernel
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_certain.py tests/test_gpu_fullframe.py tests/test_gpu_bvh.py -x -q --timeout 600 --timeout-method thread > $O/r03_42_tests.log 2>&1 || { tail -40 $O/r03_42_tests.log; exit 1; }
tail -1 $O/r03_42_tests.log
timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_42_c4.json 2> $O/r03_42_c4.err || { tail -20 $O/r03_42_c4.err; exit 1; }
tail -1 $O/r03_42_c4.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c4', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
timeout -k 10 300 python3 bench.py --config c5 --spp 16 --steps 5 --warmup 5 --no-cpu-baseline --verify-rows 4 > $O/r03_42_c5.json 2> $O/r03_42_c5.err || { tail -20 $O/r03_42_c5.err; exit 1; }
tail -1 $O/r03_42_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
timeout -k 10 300 python3 bench.py --steps 20 --warmup 8 --no-cpu-baseline --verify-rows 8 > $O/r03_42_c2.json 2> $O/r03_42_c2.err || { tail -20 $O/r03_42_c2.err; exit 1; }
tail -1 $O/r03_42_c2.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['value'], d['ms_per_step'], d['bitexact_frac_vs_oracle'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r03_42_prof_c2 -o c2 -- python3 bench.py --steps 20 --warmup 8 --no-cpu-baseline --verify-rows 0 > $O/r03_42_prof_c2.log 2>&1 || { tail -20 $O/r03_42_prof_c2.log; exit 1; }
tail -1 $O/r03_42_prof_c2.log | cut -c1-200
P="timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv"
B="python3 bench.py --steps 4 --warmup 3 --no-cpu-baseline --verify-rows 0"
$P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 -d $O/r03_42_mixa -o run -- $B > $O/r03_42_mixa.log 2>&1 || { tail -20 $O/r03_42_mixa.log; exit 1; }
$P --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $O/r03_42_mixb -o run -- $B > $O/r03_42_mixb.log 2>&1 || { tail -20 $O/r03_42_mixb.log; exit 1; }
python3 tools/pmc_mix.py $O/r03_42_mixa/run_counter_collection.csv $O/r03_42_mixb/run_counter_collection.csv c2 1 $O/r03_c2_pmc_mix_certain.json "iqpt_render_kernel C2 (certain pixels; per_iteration = per launch)" > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/r03_c2_pmc_mix_certain.json')); print('c2 mix', d['counters']['SQ_INSTS_VALU'], d['kernel_ms_profiled'], d['valu_busy_frac'], d['wave_time_split'], d['mean_waves_per_simd'])"
