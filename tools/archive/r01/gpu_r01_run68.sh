# round-1 GPU run 68: BVH work per ray on C5 (kOptStats counters)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 tools/ab_kernel.py --config c5 --spp 1 --rounds 1 --variants "prim=6951" --out gpurun_out/ab68_c5.json > gpurun_out/ab68_c5.log 2>&1 || { echo FAILED; tail -20 gpurun_out/ab68_c5.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab68_c5.json')); print(json.dumps(d['stats_default']))"
echo DONE
