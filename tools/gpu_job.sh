# r06 run 29: N = 1 with two rays per lane: the sky kernel behind (default) / ahead of the plain kernel / off (sky
# pixels in the plain kernel), alternated x3
mkdir -p gpurun_out
O=gpurun_out
R=r06_29
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
for i in 1 2 3; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/${R}_behind_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_behind_$i.json behind$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --sky-order ahead > $O/${R}_ahead_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_ahead_$i.json ahead$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --sky off > $O/${R}_off_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_off_$i.json skyoff$i
done
