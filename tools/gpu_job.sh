# r06 run 1: two rays per lane (kOptPipe): parity tests, then the default line with it on / off
mkdir -p gpurun_out
O=gpurun_out
R=r06_01
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_parity.py tests/test_gpu_overlap.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
for k in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --two-ray 1 > $O/${R}_on_$k.json 2> $O/${R}_on_$k.err || { tail -20 $O/${R}_on_$k.err; exit 1; }
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --two-ray 0 > $O/${R}_off_$k.json 2> $O/${R}_off_$k.err || { tail -20 $O/${R}_off_$k.err; exit 1; }
done
for f in $O/${R}_o*.json; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['config'].get('kernel_option_bits'), d.get('bitexact_frac_vs_oracle'))"; done
