# round-1 GPU run 31: VALU issue-rate probe, C2 instruction mix (PMC) and kernel stats of the current kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/valu_issue > gpurun_out/valu_issue.txt 2>&1 || { echo PROBE_FAILED; cat gpurun_out/valu_issue.txt; exit 1; }
cat gpurun_out/valu_issue.txt
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/pmc31a -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc31a.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/pmc31a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc31b -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc31b.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/pmc31b.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof31 -o run -- python3 bench.py --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/prof31_bench.json 2> gpurun_out/prof31_bench.err || { echo PROF_FAILED; tail -20 gpurun_out/prof31_bench.err; exit 1; }
cat gpurun_out/prof31_bench.json
find gpurun_out/pmc31a gpurun_out/pmc31b gpurun_out/prof31 -name "*.csv" | head -20
echo DONE
