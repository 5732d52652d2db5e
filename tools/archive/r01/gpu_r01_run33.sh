# round-1 GPU run 33: A/B camera matrices from LDS (kOptCamLds) on C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 9 --variants "default=2863,camlds=11055" --out gpurun_out/ab33_c2_camlds.json > gpurun_out/ab33.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab33.log; exit 1; }
head -20 gpurun_out/ab33_c2_camlds.json
echo DONE
