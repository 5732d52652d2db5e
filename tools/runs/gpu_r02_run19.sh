# round-2 run 19: executed-work counters (c2, c4, c5), FP-flavour GPU test, C4 / C5 bench lines
# priced by executed work, PMC traffic of C4 and C2 after the 16-byte accumulator store
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_fp_flavours.py -q -s --timeout 120 --timeout-method thread > gpurun_out/r02_run19_fp.log 2>&1 || exit 1
for c in c2 c4 c5; do
timeout -k 10 200 python3 tools/work_counters.py --config $c --out gpurun_out/r02_work_$c.json > gpurun_out/r02_run19_work_$c.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc19_c4_fetch -o run -- python3 bench.py --config c4 --spp 16 --steps 5 --warmup 6 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc19_c4_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc19_c4_write -o run -- python3 bench.py --config c4 --spp 16 --steps 5 --warmup 6 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc19_c4_write.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc19_c2_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc19_c2_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc19_c2_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc19_c2_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r02_pmc19_c4_fetch/run_counter_collection.csv gpurun_out/r02_pmc19_c4_write/run_counter_collection.csv c4 gpurun_out/r02_pmc_traffic_c4.json && \
python3 tools/pmc_traffic.py gpurun_out/r02_pmc19_c2_fetch/run_counter_collection.csv gpurun_out/r02_pmc19_c2_write/run_counter_collection.csv c2 gpurun_out/r02_pmc_traffic_c2.json && \
timeout -k 10 300 python3 bench.py --config c4 --spp 16 --steps 10 --warmup 6 --no-cpu-baseline --work-json gpurun_out/r02_work_c4.json --pmc-json gpurun_out/r02_pmc_traffic_c4.json > gpurun_out/r02_run19_c4.json 2> gpurun_out/r02_run19_c4.err && \
timeout -k 10 300 python3 bench.py --config c5 --spp 1 --steps 20 --warmup 6 --no-cpu-baseline --work-json gpurun_out/r02_work_c5.json --pmc-json profiles/r01_pmc_traffic_c5_v4.json > gpurun_out/r02_run19_c5.json 2> gpurun_out/r02_run19_c5.err
