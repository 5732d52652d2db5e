# r06 run 7: after the prune (chain kernel, FAN launch mode, spec queue mode archived): the whole -m gpu suite,
# smoke, the default line
mkdir -p gpurun_out
O=gpurun_out
R=r06_07
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/${R}_default.json 2> $O/${R}_default.err || { tail -20 $O/${R}_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${R}_default.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['kernel_option_bits'], d['bitexact_frac_vs_oracle'], d['lib'])"
