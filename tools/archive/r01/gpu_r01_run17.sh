# round-1 GPU run 17: tests (checkpoint), rocprof stats + PMC traffic of the current kernel, per-rank
# shares of the C3 strong-scaling split timed on one GPU
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t17.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/t17.log; exit 1; }
tail -2 gpurun_out/t17.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof17 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r17_prof.json 2> gpurun_out/r17_prof.err || { echo PROF_FAILED; tail -20 gpurun_out/r17_prof.err; exit 1; }
cat gpurun_out/r17_prof.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc17_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc17_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc17_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc17_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc17_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc17_write.log; exit 1; }
for n in 1 2 4 8; do
  rows=$(( (1080 + n - 1) / n ))
  timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 7 --crop 0,1920,0,$n,$rows --variants "default=815" --out gpurun_out/share17_n$n.json > gpurun_out/share17_n$n.log 2>&1 || { echo SHARE_FAILED $n; tail -20 gpurun_out/share17_n$n.log; exit 1; }
done
python - <<'PY'
import json
for n in (1,2,4,8):
    d=json.load(open(f"gpurun_out/share17_n{n}.json"))
    print("rank share 1/%d:" % n, d["variants"]["default"]["median_ms"], "ms")
PY
echo DONE
