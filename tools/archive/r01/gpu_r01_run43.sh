# round-1 GPU run 43: kOptCamAxis (short pitch-only camera transform): new camera tests, full GPU suite, C2 A/B, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t43a.log 2>&1 || { echo CAMTESTS_FAILED; tail -60 gpurun_out/t43a.log; exit 1; }
tail -2 gpurun_out/t43a.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t43.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t43.log; exit 1; }
tail -2 gpurun_out/t43.log
timeout -k 10 400 python tools/ab_kernel.py --config c2 --rounds 9 --variants "default=2863,axis=19247" --out gpurun_out/ab43_c2.json > gpurun_out/ab43_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab43_c2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ab43_c2.json')); print({k:(v['median_ms'],v['bitexact']) for k,v in d['variants'].items()})"
timeout -k 10 400 python bench.py > gpurun_out/b43.json 2> gpurun_out/b43.err || { echo BENCH_FAILED; tail -30 gpurun_out/b43.err; exit 1; }
cat gpurun_out/b43.json
echo DONE
