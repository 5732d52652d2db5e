# round-2 run 23: default bench line (60 s CPU baseline), rocprofv3 kernel stats of the default C2 bench,
# C5 PMC traffic before the spill work
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > gpurun_out/r02_run23_default.json 2> gpurun_out/r02_run23_default.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof23_c2 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/r02_prof23_c2.json 2> gpurun_out/r02_prof23_c2.err || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc23_c5_fetch -o run -- python3 bench.py --config c5 --spp 1 --steps 5 --warmup 6 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc23_c5_fetch.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc23_c5_write -o run -- python3 bench.py --config c5 --spp 1 --steps 5 --warmup 6 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc23_c5_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r02_pmc23_c5_fetch/run_counter_collection.csv gpurun_out/r02_pmc23_c5_write/run_counter_collection.csv c5 gpurun_out/r02_pmc_traffic_c5.json
