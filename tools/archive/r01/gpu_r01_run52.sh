# round-1 GPU run 52: sample rounds (cross-wave hand-off): rounds tests, full suite, A/B vs one round, timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rounds.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t52a.log 2>&1 || { echo ROUNDTESTS_FAILED; tail -60 gpurun_out/t52a.log; exit 1; }
tail -3 gpurun_out/t52a.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t52.log 2>&1 || { echo TESTS_FAILED; tail -60 gpurun_out/t52.log; exit 1; }
tail -2 gpurun_out/t52.log
timeout -k 10 500 python tools/ab_kernel.py --config c2 --rounds 12 --variants "one=2863@0,rounds=2863@1,axis1=19247@0,axisR=19247@1" --out gpurun_out/ab52_c2.json > gpurun_out/ab52_c2.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab52_c2.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/ab52_c2.json'))
for k,v in d['variants'].items(): print(k, v['median_ms'], v['min_ms'], v['bitexact'])
print(json.dumps(d['wave_timeline']))"
echo DONE
