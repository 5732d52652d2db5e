# round-1 GPU run 91: C5 and C4 bench lines on the final tree (same flags as run 85)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 10 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c5_v4.json --pmc-mix-json profiles/r01_c5_pmc_mix_v3.json > gpurun_out/b91_c5.json 2> gpurun_out/b91_c5.err || { echo BENCH5_FAILED; tail -20 gpurun_out/b91_c5.err; exit 1; }
cat gpurun_out/b91_c5.json
timeout -k 10 400 python3 bench.py --config c4 --spp 16 --steps 10 --warmup 3 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c4.json > gpurun_out/b91_c4.json 2> gpurun_out/b91_c4.err || { echo BENCH4_FAILED; tail -20 gpurun_out/b91_c4.err; exit 1; }
cat gpurun_out/b91_c4.json
echo DONE
