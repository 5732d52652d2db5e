# round-1 GPU run 38: near-child-first BVH traversal with an LDS stack (kOptBvhOrder): parity suite + C4/C5 A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t38.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t38.log; exit 1; }
tail -2 gpurun_out/t38.log
timeout -k 10 400 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2863,prim=6951,ord=19239,ordprim=23335" --out gpurun_out/ab38_c5.json > gpurun_out/ab38_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab38_c5.log; exit 1; }
timeout -k 10 400 python tools/ab_kernel.py --config c4 --spp 16 --rounds 3 --variants "masks=2863,prim=6951,ordprim=23335" --out gpurun_out/ab38_c4.json > gpurun_out/ab38_c4.log 2>&1 || { echo AB4_FAILED; tail -30 gpurun_out/ab38_c4.log; exit 1; }
python - <<'PY'
import json
for c in ("c5","c4"):
    d=json.load(open(f"gpurun_out/ab38_{c}.json"))
    print(c,{k:(v["median_ms"],v["bitexact"]) for k,v in d["variants"].items()})
PY
echo DONE
