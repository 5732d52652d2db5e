# round-2 run 27: production defaults now kOptScatter2 (+ kOptPrio on resident scenes): full -m gpu suite,
# smoke, default bench, C4/C5 lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_run27_tests.log 2>&1 || exit 1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_run27_smoke.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py > gpurun_out/r02_run27_default.json 2> gpurun_out/r02_run27_default.err || exit 1
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > gpurun_out/r02_run27_c4.json 2> gpurun_out/r02_run27_c4.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --no-cpu-baseline > gpurun_out/r02_run27_c5.json 2> gpurun_out/r02_run27_c5.err || exit 1
