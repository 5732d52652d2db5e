# round-1 GPU run 15: instruction mix / issue counters of the current C2 kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F --kernel-trace --output-format csv -d gpurun_out/pmc15a -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc15a.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/pmc15a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VALU --kernel-trace --output-format csv -d gpurun_out/pmc15b -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc15b.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/pmc15b.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_TRANS_F32 --kernel-trace --output-format csv -d gpurun_out/pmc15c -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc15c.log 2>&1 || { echo PMCC_FAILED; tail -20 gpurun_out/pmc15c.log; exit 1; }
echo DONE
