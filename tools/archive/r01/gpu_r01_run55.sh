# round-1 GPU run 55: stall breakdown and instruction-cache counters of the C2 kernel
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
grep -o "SQC_ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_ACTIVE_INST[A-Z_]*\|SQ_INSTS_SALU\|SQ_INST_LEVEL[A-Z_]*" gpurun_out/counters_list.txt | sort -u | tr '\n' ' '
echo
for v in 2863 19247; do
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_IFETCH SQ_WAIT_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc55a_$v -o run -- python3 tools/ab_kernel.py --config c2 --only $v --frames 2 > gpurun_out/pmc55a_$v.log 2>&1 || { echo PMC_FAILED $v; tail -20 gpurun_out/pmc55a_$v.log; exit 1; }
done
echo DONE
