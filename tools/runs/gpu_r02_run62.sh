# round-2 run 62: chain kernel stops tracing slots the chain has passed (dead while in flight): chain +
# overlap + split tests, then A/B shares (tools/split_share.py, chain mode, N = 1/2/4/8) against a library
# built with -DIQPT_CHAIN_NO_ABORT, alternating, and the bench's N = 4 / 8 shares through the gather step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_run62_tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python3 tools/split_share.py --ns 1,2,4,8 --modes chain --launches 10 --out gpurun_out/r02_run62_abort_$r.json > gpurun_out/r02_run62_skip_$r.log 2>&1 || exit 1
  timeout -k 10 200 python3 tools/split_share.py --ns 1,2,4,8 --modes chain --launches 10 --lib tools/libiqpt_noabort.so --out gpurun_out/r02_run62_noabort_$r.json > gpurun_out/r02_run62_noskip_$r.log 2>&1 || exit 1
done
for n in 4 8; do
  timeout -k 10 200 python3 bench.py --self-gather --share-of $n --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r02_run62_share$n.json 2> gpurun_out/r02_run62_share$n.err || exit 1
done
