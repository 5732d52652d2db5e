# round-1 GPU run 37: BVH with normal cones (growth scaled by 1e-6 / D): parity suite, C4/C5 full-frame A/B, bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t37.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t37.log; exit 1; }
tail -2 gpurun_out/t37.log
timeout -k 10 400 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --variants "masks=2863,prim=6951" --out gpurun_out/ab37_c5_full.json > gpurun_out/ab37_c5.log 2>&1 || { echo AB5_FAILED; tail -30 gpurun_out/ab37_c5.log; exit 1; }
timeout -k 10 400 python tools/ab_kernel.py --config c4 --spp 16 --rounds 3 --variants "masks=2863,prim=6951" --out gpurun_out/ab37_c4_full.json > gpurun_out/ab37_c4.log 2>&1 || { echo AB4_FAILED; tail -30 gpurun_out/ab37_c4.log; exit 1; }
python - <<'PY'
import json
for c in ("c5","c4"):
    d=json.load(open(f"gpurun_out/ab37_{c}_full.json"))
    print(c,{k:(v["median_ms"],v["bitexact"]) for k,v in d["variants"].items()})
PY
timeout -k 10 400 python bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r37_bench_c5.json 2> gpurun_out/r37_bench_c5.err || { echo BENCH5_FAILED; tail -30 gpurun_out/r37_bench_c5.err; exit 1; }
cat gpurun_out/r37_bench_c5.json
timeout -k 10 400 python bench.py --config c4 --spp 16 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r37_bench_c4.json 2> gpurun_out/r37_bench_c4.err || { echo BENCH4_FAILED; tail -30 gpurun_out/r37_bench_c4.err; exit 1; }
cat gpurun_out/r37_bench_c4.json
echo DONE
