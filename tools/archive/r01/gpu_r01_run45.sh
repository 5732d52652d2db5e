# round-1 GPU run 45: camera-axis formulations A/B (packed vs scalar) against the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_camera.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t45a.log 2>&1 || { echo CAMTESTS_FAILED; tail -60 gpurun_out/t45a.log; exit 1; }
tail -1 gpurun_out/t45a.log
timeout -k 10 500 python tools/ab_kernel.py --config c2 --rounds 11 --variants "default=2863,axis=19247,axisS=52015" --out gpurun_out/ab45_c2.json > gpurun_out/ab45_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab45_c2.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/ab45_c2.json')); print({k:(v['median_ms'],v['min_ms'],v['bitexact']) for k,v in d['variants'].items()})"
echo DONE
