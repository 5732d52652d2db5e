# round-2 run 35: kernel traces of chain launches (the chain kernel and the plain kernel beside it), N = 8 and 2
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 8 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r02_run35_trace_n$n -o run -- python3 tools/split_share.py --modes chain --ns $n --chain-waves 16 --launches 6 --warm 1 > gpurun_out/r02_run35_n$n.log 2>&1 || exit 1
done
