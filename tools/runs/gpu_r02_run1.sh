set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run1_pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --cpu-seconds 10 > gpurun_out/r02_run1_bench.json 2> gpurun_out/r02_run1_bench.err && \
lscpu > gpurun_out/r02_lscpu.txt 2>&1 && nproc > gpurun_out/r02_nproc.txt && python -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))" >> gpurun_out/r02_nproc.txt
