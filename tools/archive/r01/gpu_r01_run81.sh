# round-1 GPU run 81: full GPU suite + smoke, then C5 profile refresh after spheres-first (PMC mix,
# HBM traffic, bench line), C4 bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t81.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t81.log; exit 1; }
tail -2 gpurun_out/t81.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke81.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke81.log; exit 1; }
tail -2 gpurun_out/smoke81.log
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/p81_mixa -o run -- python3 tools/ab_kernel.py --config c5 --spp 1 --only 6959 --frames 2 > gpurun_out/p81_mixa.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/p81_mixa.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/p81_mixb -o run -- python3 tools/ab_kernel.py --config c5 --spp 1 --only 6959 --frames 2 > gpurun_out/p81_mixb.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/p81_mixb.log; exit 1; }
python3 tools/pmc_mix.py gpurun_out/p81_mixa/run_counter_collection.csv gpurun_out/p81_mixb/run_counter_collection.csv c5 1 gpurun_out/p81_mix_c5.json "iqpt_render_kernel<8,true,6959>"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/p81_fetch -o run -- python3 bench.py --config c5 --spp 1 --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0 > gpurun_out/p81_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/p81_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p81_write -o run -- python3 bench.py --config c5 --spp 1 --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0 > gpurun_out/p81_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/p81_write.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/p81_fetch/run_counter_collection.csv gpurun_out/p81_write/run_counter_collection.csv c5 gpurun_out/p81_traffic_c5.json
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 10 --warmup 3 --no-cpu-baseline --pmc-json gpurun_out/p81_traffic_c5.json --pmc-mix-json gpurun_out/p81_mix_c5.json > gpurun_out/b81_c5.json 2> gpurun_out/b81_c5.err || { echo BENCH5_FAILED; tail -20 gpurun_out/b81_c5.err; exit 1; }
cat gpurun_out/b81_c5.json
timeout -k 10 400 python3 bench.py --config c4 --spp 16 --steps 10 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c4.json > gpurun_out/b81_c4.json 2> gpurun_out/b81_c4.err || { echo BENCH4_FAILED; tail -20 gpurun_out/b81_c4.err; exit 1; }
cat gpurun_out/b81_c4.json
echo DONE
