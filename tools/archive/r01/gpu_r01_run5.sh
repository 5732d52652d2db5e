set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
# C2 variant set on the resident path
timeout -k 10 600 python tools/ab_kernel.py --config c2 --rounds 7 --variants "none=0,ca=3,cas=35,camtf=19" --out gpurun_out/ab5_c2.json > gpurun_out/ab5_c2.log 2>&1 || { echo AB1_FAILED; tail -30 gpurun_out/ab5_c2.log; exit 1; }
# C4 crop (10k triangles streamed through LDS)
timeout -k 10 600 python tools/ab_kernel.py --config c4 --spp 2 --rounds 3 --crop 0,1920,400,1,256 --variants "none=0,ca=3,camtf=19,camtfdef=23,cadef=7" --out gpurun_out/ab5_c4.json > gpurun_out/ab5_c4.log 2>&1 || { echo AB2_FAILED; tail -30 gpurun_out/ab5_c4.log; exit 1; }
# C5 crop (50k tris + 1k spheres)
timeout -k 10 600 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --crop 0,3840,1000,1,64 --variants "none=0,ca=3,camtf=19,camtfdef=23,cadef=7" --out gpurun_out/ab5_c5.json > gpurun_out/ab5_c5.log 2>&1 || { echo AB3_FAILED; tail -30 gpurun_out/ab5_c5.log; exit 1; }
python - <<'PY'
import json
for n in ("c2","c4","c5"):
    d=json.load(open(f"gpurun_out/ab5_{n}.json"))
    print(n, {k:(v["median_ms"], v["vs_default"], v["bitexact"]) for k,v in d["variants"].items()})
    print("  stats", d["stats_default"])
PY
# hardware counters on the C2 'ca' variant
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH --kernel-trace --output-format csv -d gpurun_out/pmc5a -o run -- python3 tools/ab_kernel.py --config c2 --only 3 --frames 2 > gpurun_out/pmc5a.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/pmc5a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc5b -o run -- python3 tools/ab_kernel.py --config c2 --only 3 --frames 2 > gpurun_out/pmc5b.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/pmc5b.log; exit 1; }
echo DONE
