# r06 run 44: the committed tree (kernel_sha16 3a8d33396bae8753, bench.py's 100-step default): the whole -m gpu
# suite and smoke, as the driver runs them at round end
mkdir -p gpurun_out
O=gpurun_out
R=r06_44
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
