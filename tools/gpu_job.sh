# r03 run 10: spec with self-contained run records: exactness, statistics, kernel trace at N = 8
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_fan.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_run10_tests.log 2>&1 || { tail -40 gpurun_out/r03_run10_tests.log; exit 1; }
tail -2 gpurun_out/r03_run10_tests.log
timeout -k 10 400 python -u tools/split_share.py --modes spec,chain,fan --ns 8,4,2,1 --launches 6 --out gpurun_out/r03_share_v6.json > gpurun_out/r03_run10_share.log 2>&1 || { tail -30 gpurun_out/r03_run10_share.log; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/r03_share_v6.json'))
for r in d['rows']: print({k:(round(v,3) if isinstance(v,float) else v) for k,v in r.items() if k!='split_info' and 'min' not in k})"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03_prof10_spec8 -o run -- python3 tools/split_share.py --modes spec --ns 8 --launches 4 --warm 2 > gpurun_out/r03_run10_prof.log 2>&1 || { tail -20 gpurun_out/r03_run10_prof.log; exit 1; }
python3 - <<'PY'
import csv
rows=[r for r in csv.DictReader(open('gpurun_out/r03_prof10_spec8/run_kernel_trace.csv')) if 'iqpt_' in r['Kernel_Name'] or 'fill' in r['Kernel_Name']]
rows.sort(key=lambda r:int(r['Start_Timestamp']))
t0=int(rows[-8]['Start_Timestamp'])
for r in rows[-8:]:
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    print(r['Kernel_Name'][:50], round(s,1), round(e-s,1))
PY
