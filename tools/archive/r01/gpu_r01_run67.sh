# round-1 GPU run 67: full GPU suite after the list changes; C4 / C5 HBM traffic (PMC) and bench lines with it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t67.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t67.log; exit 1; }
tail -2 gpurun_out/t67.log
for c in c4 c5; do
  if [ $c = c4 ]; then spp=16; else spp=1; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/p67_${c}_fetch -o run -- python3 bench.py --config $c --spp $spp --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/p67_${c}_fetch.log 2>&1 || { echo PMC1_FAILED $c; tail -20 gpurun_out/p67_${c}_fetch.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/p67_${c}_write -o run -- python3 bench.py --config $c --spp $spp --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 > gpurun_out/p67_${c}_write.log 2>&1 || { echo PMC2_FAILED $c; tail -20 gpurun_out/p67_${c}_write.log; exit 1; }
  python3 tools/pmc_traffic.py gpurun_out/p67_${c}_fetch/run_counter_collection.csv gpurun_out/p67_${c}_write/run_counter_collection.csv $c gpurun_out/p67_${c}_traffic.json
  timeout -k 10 400 python3 bench.py --config $c --spp $spp --steps 5 --warmup 3 --no-cpu-baseline --pmc-json gpurun_out/p67_${c}_traffic.json > gpurun_out/b67_$c.json 2> gpurun_out/b67_$c.err || { echo BENCH_FAILED $c; tail -20 gpurun_out/b67_$c.err; exit 1; }
  cat gpurun_out/b67_$c.json
done
echo DONE
