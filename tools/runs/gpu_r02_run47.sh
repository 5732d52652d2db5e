# round-2 run 47: profiles of the current tree: rocprofv3 kernel stats of the default C2 bench, C2 PMC traffic
# (separate FETCH / WRITE passes), C4 and C5 bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_prof47_c2 -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/r02_prof47_c2.json 2> gpurun_out/r02_prof47_c2.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc47_c2_fetch -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc47_c2_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/r02_pmc47_c2_write -o run -- python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --verify-rows 0 > gpurun_out/r02_pmc47_c2_write.log 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/r02_pmc47_c2_fetch/run_counter_collection.csv gpurun_out/r02_pmc47_c2_write/run_counter_collection.csv c2 gpurun_out/r02_pmc_traffic_c2_v2.json || exit 1
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/r02_run47_c4.json 2> gpurun_out/r02_run47_c4.err || exit 1
# (the C5 line, 20 steps of the default 1024 spp, ran silent past the 180-s limit: run 48 takes 16 spp x 5 steps)
