# round-2 run 54: (rejected, reverted) candidate lists sorted by the pairs' t lower bounds with an early exit: full -m gpu suite, C4 and
# C5 bench lines with and without (--list-order index), alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run54_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 bench.py --config c4 --spp 64 --steps 10 --no-cpu-baseline > gpurun_out/r02_run54_c4_bound_$r.json 2>/dev/null || exit 1
  timeout -k 10 200 python3 bench.py --config c4 --spp 64 --steps 10 --no-cpu-baseline --list-order index > gpurun_out/r02_run54_c4_index_$r.json 2>/dev/null || exit 1
done
timeout -k 10 200 python3 bench.py --config c5 --spp 16 --steps 5 --no-cpu-baseline --verify-rows 4 > gpurun_out/r02_run54_c5_bound.json 2>/dev/null || exit 1
timeout -k 10 200 python3 bench.py --config c5 --spp 16 --steps 5 --no-cpu-baseline --verify-rows 4 --list-order index > gpurun_out/r02_run54_c5_index.json 2>/dev/null || exit 1
