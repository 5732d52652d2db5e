# round-1 GPU run 49: busy/clock counters of default vs camera-axis variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2863 19247; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/pmc49_$v -o run -- python3 tools/ab_kernel.py --config c2 --only $v --frames 4 > gpurun_out/pmc49_$v.log 2>&1 || { echo PMC_FAILED $v; tail -20 gpurun_out/pmc49_$v.log; exit 1; }
done
echo DONE
