set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run18_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-seconds 5 > gpurun_out/r02_run18_bench.json 2> gpurun_out/r02_run18_bench.err && \
timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --one-device --no-cpu-baseline --steps 5 > gpurun_out/r02_run18_bench2.json 2> gpurun_out/r02_run18_bench2.err
