# round-1 GPU run 71: C5 bench line after the no-batch BVH-primary kernel (with its traffic file)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/p71_fetch -o run -- python3 bench.py --config c5 --spp 1 --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/p71_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/p71_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p71_write -o run -- python3 bench.py --config c5 --spp 1 --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/p71_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/p71_write.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/p71_fetch/run_counter_collection.csv gpurun_out/p71_write/run_counter_collection.csv c5 gpurun_out/p71_c5_traffic.json
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 5 --warmup 3 --no-cpu-baseline --pmc-json gpurun_out/p71_c5_traffic.json > gpurun_out/b71_c5.json 2> gpurun_out/b71_c5.err || { echo BENCH_FAILED; tail -20 gpurun_out/b71_c5.err; exit 1; }
cat gpurun_out/b71_c5.json
echo DONE
