# r06 run 6: plain-kernel wave timelines with per-phase cycles (two rays on / off; full frame overlapped, sphere crop)
mkdir -p gpurun_out
O=gpurun_out
R=r06_06
export TMPDIR=/tmp
for t in 1 0; do
  timeout -k 10 300 python3 tools/wave_timeline.py --two-ray $t --out $O/${R}_wt_full_t$t.json > $O/${R}_wt_full_t$t.log 2>&1 || { tail -20 $O/${R}_wt_full_t$t.log; exit 1; }
  timeout -k 10 300 python3 tools/wave_timeline.py --two-ray $t --overlap 0 --crop 760,1160,480,96 --out $O/${R}_wt_crop_t$t.json > $O/${R}_wt_crop_t$t.log 2>&1 || { tail -20 $O/${R}_wt_crop_t$t.log; exit 1; }
done
for f in $O/${R}_wt_*.json; do python3 -c "
import json; d=json.load(open('$f'))
t=d['longest_5pct']
print('$f', d['kernel_ms'], 'iters', t['iters']['50'], 'us/iter', t['us_per_iter']['50'], {k: v['50'] for k, v in t['cycles_per_iter'].items()})"; done
