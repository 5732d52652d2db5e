set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in sphere_tile wall_tile; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/r02_pmc11a_$c -o run -- python3 tools/lone_wave.py - $c > gpurun_out/r02_pmc11a_$c.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VALU --kernel-trace --output-format csv -d gpurun_out/r02_pmc11b_$c -o run -- python3 tools/lone_wave.py - $c > gpurun_out/r02_pmc11b_$c.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_IFETCH --kernel-trace --output-format csv -d gpurun_out/r02_pmc11c_$c -o run -- python3 tools/lone_wave.py - $c > gpurun_out/r02_pmc11c_$c.log 2>&1 || exit 1
done
