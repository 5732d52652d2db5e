# round-2 run 51: (rejected, reverted) unit colour shortcut for camera rays ending on an emissive triangle (no clamp / division):
# full -m gpu suite, smoke, three default benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run51_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run51_smoke.log 2>&1 || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python3 bench.py --steps 40 --no-cpu-baseline --verify-rows 8 > gpurun_out/r02_run51_b$r.json 2>/dev/null || exit 1
done
timeout -k 10 400 python3 tools/split_share.py --modes plain,chain --ns 1,2,4,8 --out gpurun_out/r02_run51_share.json > gpurun_out/r02_run51_share.log 2>&1 || exit 1
