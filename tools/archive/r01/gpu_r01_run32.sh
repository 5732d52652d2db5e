# round-1 GPU run 32: PC sampling (host trap) of the C2 render kernel: where the issue slots go
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/rocprof_avail.txt 2>&1 || true
grep -i -A12 "pc sampling\|pc_sampling" gpurun_out/rocprof_avail.txt | head -40
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 50 --output-format csv -d gpurun_out/pcs32 -o run -- python3 tools/ab_kernel.py --config c2 --only default --frames 4 > gpurun_out/pcs32.log 2>&1 || { echo PCS_FAILED; tail -30 gpurun_out/pcs32.log; exit 1; }
tail -5 gpurun_out/pcs32.log
find gpurun_out/pcs32 -type f | head; 
echo DONE
