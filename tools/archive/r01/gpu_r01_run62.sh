# round-1 GPU run 62: C3 strong-scaling shares of the current kernel (row r, r+N, ... of the C2 frame on one GPU)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 1 2 4 8; do
  rows=$((1080 / n))
  timeout -k 10 300 python tools/ab_kernel.py --config c2 --rounds 7 --crop 0,1920,0,$n,$rows --variants "default=2863" --out gpurun_out/share62_n$n.json > gpurun_out/share62_n$n.log 2>&1 || { echo SHARE_FAILED $n; tail -20 gpurun_out/share62_n$n.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/share62_n$n.json')); print($n, d['variants']['default']['median_ms'], json.dumps(d['wave_timeline']['end_us_pct']) if d.get('wave_timeline') else '')"
done
echo DONE
