# r06 run 9: per-pixel candidate masks over the streamed tile lists (C4): parity tests, C4 line with masks on / off
mkdir -p gpurun_out
O=gpurun_out
R=r06_09
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pixel_masks.py tests/test_gpu_fullframe.py tests/test_gpu_bvh.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], r.get('frac'), d['config'].get('kernel_option_bits'))"; }
for m in 1 0 1; do
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --pixel-masks $m > $O/${R}_c4_m$m.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4_m$m.json c4_masks$m
done
