# round-1 GPU run 53: after reverting sample rounds: GPU suite, default vs camera-axis A/B, 20-frame averages
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t53.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t53.log; exit 1; }
tail -2 gpurun_out/t53.log
: > gpurun_out/r53.txt
for r in 1 2; do
for v in 2863 19247; do
timeout -k 10 120 python3 tools/ab_kernel.py --config c2 --only $v --frames 20 >> gpurun_out/r53.txt 2> gpurun_out/r53.err || { echo FAILED $v; tail -20 gpurun_out/r53.err; exit 1; }
done
done
cat gpurun_out/r53.txt
echo DONE
