# r03 run 54: spec plan lane cap A/B at N = 8 / 4 / 2 (tools/ab_spec_cap.py), after the spec tests
mkdir -p gpurun_out
O=gpurun_out
R=r03_54
timeout -k 10 400 python -u -m pytest tests/test_gpu_spec.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 400 python3 -u tools/ab_spec_cap.py --ns 8,4,2 --caps 0.97,0.5,0.75,1.25,2.0,4.0 --rounds 2 --out $O/${R}_spec_cap.json > $O/${R}_spec_cap.log 2>&1 || { tail -20 $O/${R}_spec_cap.log; exit 1; }
cat $O/${R}_spec_cap.log
