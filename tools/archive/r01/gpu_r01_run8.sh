set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 9 --variants "pair=39,pairlb5=47,nb=103,nblb5=111,nopair=35,nopairlb6=51" --out gpurun_out/ab8_c2.json > gpurun_out/ab8_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab8_c2.log; exit 1; }
timeout -k 10 300 python tools/ab_kernel.py --config c4 --spp 2 --rounds 3 --crop 0,1920,400,1,256 --variants "pair=39,pairlb5=47,nopair=35" --out gpurun_out/ab8_c4.json > gpurun_out/ab8_c4.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab8_c4.log; exit 1; }
python - <<'PY'
import json
for n in ("c2","c4"):
    d=json.load(open(f"gpurun_out/ab8_{n}.json"))
    print(n, {k:(v["median_ms"], v["vs_default"], v["bitexact"]) for k,v in d["variants"].items()})
PY
