# round-2 run 49: stream-ordered per-step frame gather (no host sync in the step): one-rank nccl process group
# through the gather path (stream-ordered and blocking), the multi-rank bench tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --self-gather --steps 20 --no-cpu-baseline > gpurun_out/r02_run49_selfgather.json 2> gpurun_out/r02_run49_selfgather.err || exit 1
timeout -k 10 200 python3 bench.py --self-gather --gather-sync --steps 20 --no-cpu-baseline > gpurun_out/r02_run49_selfgather_sync.json 2> gpurun_out/r02_run49_selfgather_sync.err || exit 1
timeout -k 10 200 python3 bench.py --self-gather --split chain --steps 20 --no-cpu-baseline > gpurun_out/r02_run49_selfgather_chain.json 2> gpurun_out/r02_run49_selfgather_chain.err || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_multirank.py tests/test_capi.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run49_tests.log 2>&1 || exit 1
