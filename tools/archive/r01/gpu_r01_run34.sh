# round-1 GPU run 34: C2 wave-level work counters (pair tests per iteration, full-loop iterations)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 1 --variants "default=2863" --out gpurun_out/ab34_c2_stats.json > gpurun_out/ab34.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab34.log; exit 1; }
cat gpurun_out/ab34_c2_stats.json
echo DONE
