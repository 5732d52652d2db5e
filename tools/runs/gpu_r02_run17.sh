set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
n=8
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM --kernel-trace --output-format csv -d gpurun_out/r02_pmc17a -o run -- python3 tools/split_share.py --ns $n --modes plain --knobs 65535:16 --launches 2 --warm 1 > gpurun_out/r02_pmc17a.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VALU --kernel-trace --output-format csv -d gpurun_out/r02_pmc17b -o run -- python3 tools/split_share.py --ns $n --modes plain --knobs 65535:16 --launches 2 --warm 1 > gpurun_out/r02_pmc17b.log 2>&1
