# r06 run 14: compact per-pixel masks (lists up to 1,024 entries; iqpt_anyhit_kernel up to 512): parity tests, C4 line
mkdir -p gpurun_out
O=gpurun_out
R=r06_14
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/list_stats.py --config c4 > $O/${R}_c4_lists.json 2>&1 || { tail -20 $O/${R}_c4_lists.json; exit 1; }
cat $O/${R}_c4_lists.json
timeout -k 10 900 python -u -m pytest tests/test_gpu_pixel_masks.py tests/test_gpu_fullframe.py tests/test_gpu_bvh.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'), d['config'].get('launch_mode'))"; }
for m in 2 1 2; do
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --pixel-masks $m > $O/${R}_c4_m$m.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4_m$m.json c4_mode$m
done
