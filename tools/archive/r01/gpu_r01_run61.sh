# round-1 GPU run 61: profile refresh of the current C2 kernel: HBM traffic (separate FETCH/WRITE passes),
# instruction mix + wave-time split, rocprofv3 kernel stats of 60 bench steps, bench with CPU baseline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/p61_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/p61_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/p61_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p61_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/p61_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/p61_write.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/p61_fetch/run_counter_collection.csv gpurun_out/p61_write/run_counter_collection.csv c2 gpurun_out/p61_traffic.json
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/p61_mixa -o run -- python3 tools/ab_kernel.py --config c2 --only 2863 --frames 2 > gpurun_out/p61_mixa.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/p61_mixa.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/p61_mixb -o run -- python3 tools/ab_kernel.py --config c2 --only 2863 --frames 2 > gpurun_out/p61_mixb.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/p61_mixb.log; exit 1; }
python3 tools/pmc_mix.py gpurun_out/p61_mixa/run_counter_collection.csv gpurun_out/p61_mixb/run_counter_collection.csv c2 2188285 gpurun_out/p61_mix.json "iqpt_render_kernel<8,false,2863>"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p61_stats -o run -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline --pmc-json gpurun_out/p61_traffic.json --pmc-mix-json gpurun_out/p61_mix.json > gpurun_out/p61_stats_bench.json 2> gpurun_out/p61_stats_bench.err || { echo PROF_FAILED; tail -20 gpurun_out/p61_stats_bench.err; exit 1; }
cat gpurun_out/p61_stats_bench.json
timeout -k 10 400 python3 bench.py --pmc-json gpurun_out/p61_traffic.json --pmc-mix-json gpurun_out/p61_mix.json > gpurun_out/p61_bench.json 2> gpurun_out/p61_bench.err || { echo BENCH_FAILED; tail -20 gpurun_out/p61_bench.err; exit 1; }
cat gpurun_out/p61_bench.json
echo DONE
