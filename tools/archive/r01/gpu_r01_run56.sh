# round-1 GPU run 56: refill frequency (kOptStats) on C2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab_kernel.py --config c2 --rounds 2 --variants "default=2863" --out gpurun_out/ab56.json > gpurun_out/ab56.log 2>&1 || { echo FAILED; tail -20 gpurun_out/ab56.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab56.json')); print(json.dumps(d['stats_default']))"
echo DONE
