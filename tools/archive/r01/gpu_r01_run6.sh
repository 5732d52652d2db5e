set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t6.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t6.log; exit 1; }
tail -2 gpurun_out/t6.log
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
timeout -k 10 600 python tools/ab_kernel.py --config c2 --rounds 9 --out gpurun_out/ab6_c2.json > gpurun_out/ab6_c2.log 2>&1 || { echo AB1_FAILED; tail -30 gpurun_out/ab6_c2.log; exit 1; }
timeout -k 10 600 python tools/ab_kernel.py --config c4 --spp 2 --rounds 3 --crop 0,1920,400,1,256 --variants "default=39,-pair=35,none=0" --out gpurun_out/ab6_c4.json > gpurun_out/ab6_c4.log 2>&1 || { echo AB2_FAILED; tail -30 gpurun_out/ab6_c4.log; exit 1; }
python - <<'PY'
import json
for n in ("c2","c4"):
    d=json.load(open(f"gpurun_out/ab6_{n}.json"))
    print(n, {k:(v["median_ms"], v["vs_default"], v["bitexact"]) for k,v in d["variants"].items()})
    print("  stats", d["stats_default"])
PY
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F --kernel-trace --output-format csv -d gpurun_out/pmc6a -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc6a.log 2>&1 || { echo PMCA_FAILED; tail -20 gpurun_out/pmc6a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INST_CYCLES_VALU --kernel-trace --output-format csv -d gpurun_out/pmc6b -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 2 > gpurun_out/pmc6b.log 2>&1 || { echo PMCB_FAILED; tail -20 gpurun_out/pmc6b.log; exit 1; }
echo DONE
