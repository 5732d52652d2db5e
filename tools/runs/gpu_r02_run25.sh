# round-2 run 25: A/B of VALU issue priority for critical-path waves (kOptPrio) on C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ab_kernel.py --config c2 --rounds 11 --variants default=2863,prio=133935,prioexp=166703 --out gpurun_out/r02_ab_prio.json > gpurun_out/r02_run25.log 2>&1 && \
timeout -k 10 300 python -u tools/ab_kernel.py --config c2 --rounds 1 --variants default=2863 --stats-opt 133935 --out gpurun_out/r02_ab_prio_stats.json >> gpurun_out/r02_run25.log 2>&1
