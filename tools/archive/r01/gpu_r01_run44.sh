# round-1 GPU run 44: packed running mean (+ mean_tiny guard), uniform-tile masks, launches split at the table size
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_materials.py tests/test_gpu_camera.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t44a.log 2>&1 || { echo NEWTESTS_FAILED; tail -60 gpurun_out/t44a.log; exit 1; }
tail -2 gpurun_out/t44a.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t44.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t44.log; exit 1; }
tail -2 gpurun_out/t44.log
timeout -k 10 400 python tools/ab_kernel.py --config c2 --rounds 9 --variants "default=2863,axis=19247" --out gpurun_out/ab44_c2.json > gpurun_out/ab44_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab44_c2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ab44_c2.json')); print({k:(v['median_ms'],v['bitexact']) for k,v in d['variants'].items()})"
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/b44.json 2> gpurun_out/b44.err || { echo BENCH_FAILED; tail -30 gpurun_out/b44.err; exit 1; }
cat gpurun_out/b44.json
echo DONE
