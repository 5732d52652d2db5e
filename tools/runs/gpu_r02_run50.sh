# round-2 run 50: C2 instruction mix / wave-time split of the current render kernel (PMC passes; rocprofv3 runs the
# launches one at a time while it collects counters)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/r02_mix50a -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_mix50a.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/r02_mix50b -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_mix50b.log 2>&1 || exit 1
python3 tools/pmc_mix.py gpurun_out/r02_mix50a/run_counter_collection.csv gpurun_out/r02_mix50b/run_counter_collection.csv c2 1 gpurun_out/r02_c2_pmc_mix_v5.json "iqpt_render_kernel (overlap + short camera)" || exit 1
