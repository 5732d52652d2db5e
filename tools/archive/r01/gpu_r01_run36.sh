# round-1 GPU run 36: C2 timing ablations (camera ray / intersection / running mean removed; not exact)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 9 --variants "default=2863,d0=11055#0,d1=11055#1,d2=11055#2,d4=11055#4,d3=11055#3,d7=11055#7" --out gpurun_out/ab36_c2_ablate.json > gpurun_out/ab36.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab36.log; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/ab36_c2_ablate.json"))
print({k:(v["median_ms"],v["bitexact"]) for k,v in d["variants"].items()})
PY
echo DONE
