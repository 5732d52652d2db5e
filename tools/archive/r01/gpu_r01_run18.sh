# round-1 GPU run 18: LDS scatter stack + per-pixel mask slot + LDS sphere lookup: tests, bench,
# per-rank shares of C3, C4/C5 crops
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t18.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t18.log; exit 1; }
tail -2 gpurun_out/t18.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r18_bench.json 2> gpurun_out/r18_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r18_bench.err; exit 1; }
cat gpurun_out/r18_bench.json
for n in 1 2 4 8; do
  rows=$(( (1080 + n - 1) / n ))
  timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 7 --crop 0,1920,0,$n,$rows --variants "default=815" --out gpurun_out/share18_n$n.json > gpurun_out/share18_n$n.log 2>&1 || { echo SHARE_FAILED $n; tail -20 gpurun_out/share18_n$n.log; exit 1; }
done
timeout -k 10 600 python tools/ab_kernel.py --config c4 --spp 2 --rounds 3 --crop 0,1920,400,1,256 --variants "default=815,nocull=303" --out gpurun_out/ab18_c4.json > gpurun_out/ab18_c4.log 2>&1 || { echo AB2_FAILED; tail -30 gpurun_out/ab18_c4.log; exit 1; }
timeout -k 10 600 python tools/ab_kernel.py --config c5 --spp 1 --rounds 3 --crop 0,3840,1000,1,64 --variants "default=815,nocull=303" --out gpurun_out/ab18_c5.json > gpurun_out/ab18_c5.log 2>&1 || { echo AB3_FAILED; tail -30 gpurun_out/ab18_c5.log; exit 1; }
python - <<'PY'
import json
for n in (1,2,4,8):
    d=json.load(open(f"gpurun_out/share18_n{n}.json"))
    print("rank share 1/%d:" % n, d["variants"]["default"]["median_ms"], "ms")
for n in ("c4","c5"):
    d=json.load(open(f"gpurun_out/ab18_{n}.json"))
    print(n, {k:(v["median_ms"], v["vs_default"], v["bitexact"]) for k,v in d["variants"].items()})
PY
echo DONE
