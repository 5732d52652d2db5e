# round-1 GPU run 35: batched pixel turnover (refill when >= k lanes idle): parity suite + C2/C4/C5 A/B over k
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t35.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t35.log; exit 1; }
tail -2 gpurun_out/t35.log
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 9 --variants "k1=2863@1,k4=2863@4,k8=2863@8,k12=2863@12,k16=2863@16,k24=2863@24" --out gpurun_out/ab35_c2_refill.json > gpurun_out/ab35.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab35.log; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/ab35_c2_refill.json"))
print({k:(v["median_ms"],v["bitexact"]) for k,v in d["variants"].items()})
PY
timeout -k 10 300 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "k1=2863@1,k8=2863@8,k16=2863@16" --out gpurun_out/ab35_c5_refill.json > gpurun_out/ab35_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab35_c5.log; exit 1; }
timeout -k 10 300 python tools/ab_kernel.py --config c4 --spp 16 --rounds 3 --variants "k1=2863@1,k8=2863@8,k16=2863@16" --out gpurun_out/ab35_c4_refill.json > gpurun_out/ab35_c4.log 2>&1 || { echo AB4_FAILED; tail -30 gpurun_out/ab35_c4.log; exit 1; }
python - <<'PY'
import json
for c in ("c5","c4"):
    d=json.load(open(f"gpurun_out/ab35_{c}_refill.json"))
    print(c,{k:(v["median_ms"],v["bitexact"]) for k,v in d["variants"].items()})
PY
echo DONE
