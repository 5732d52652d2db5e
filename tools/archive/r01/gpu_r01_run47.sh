# round-1 GPU run 47: instruction mix (PMC) of default / camera-axis variants
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 2863 19247 52015; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc47_$v -o run -- python3 tools/ab_kernel.py --config c2 --only $v --frames 2 > gpurun_out/pmc47_$v.log 2>&1 || { echo PMC_FAILED $v; tail -20 gpurun_out/pmc47_$v.log; exit 1; }
done
find gpurun_out/pmc47_* -name "*counter_collection*.csv"
echo DONE
