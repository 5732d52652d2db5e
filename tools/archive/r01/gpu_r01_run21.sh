# round-1 GPU run 21: rocprof stats + PMC traffic + instruction mix of the current C2 kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof21 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r21_prof.json 2> gpurun_out/r21_prof.err || { echo PROF_FAILED; tail -20 gpurun_out/r21_prof.err; exit 1; }
cat gpurun_out/r21_prof.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc21_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc21_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc21_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc21_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc21_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc21_write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/pmc21a -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc21a.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/pmc21a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc21b -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc21b.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/pmc21b.log; exit 1; }
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 3 --variants "default=815" --out gpurun_out/ab21_stats.json > gpurun_out/ab21_stats.log 2>&1 || { echo STATS_FAILED; tail -20 gpurun_out/ab21_stats.log; exit 1; }
echo DONE
