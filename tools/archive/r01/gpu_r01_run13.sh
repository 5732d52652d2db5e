# round-1 GPU run 13: fast exact division — exhaustive/randomised proof, parity, A/B, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/fastdiv_check 4 > gpurun_out/fastdiv13.txt 2>&1 || { echo FASTDIV_FAILED; cat gpurun_out/fastdiv13.txt; exit 1; }
cat gpurun_out/fastdiv13.txt
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t13.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t13.log; exit 1; }
tail -2 gpurun_out/t13.log
timeout -k 10 600 python tools/ab_kernel.py --config c2 --rounds 9 --variants "default=303,nofast=47" --out gpurun_out/ab13_c2.json > gpurun_out/ab13_c2.log 2>&1 || { echo AB1_FAILED; tail -30 gpurun_out/ab13_c2.log; exit 1; }
timeout -k 10 600 python tools/ab_kernel.py --config c4 --spp 2 --rounds 3 --crop 0,1920,400,1,256 --variants "default=303,nofast=47" --out gpurun_out/ab13_c4.json > gpurun_out/ab13_c4.log 2>&1 || { echo AB2_FAILED; tail -30 gpurun_out/ab13_c4.log; exit 1; }
python - <<'PY'
import json
for n in ("c2","c4"):
    d=json.load(open(f"gpurun_out/ab13_{n}.json"))
    print(n, {k:(v["median_ms"], v["vs_default"], v["bitexact"]) for k,v in d["variants"].items()})
PY
timeout -k 10 400 python bench.py > gpurun_out/r13_bench.json 2> gpurun_out/r13_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r13_bench.err; exit 1; }
cat gpurun_out/r13_bench.json
echo DONE
