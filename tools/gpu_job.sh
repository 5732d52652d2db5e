# r05 run 17: any-hit as variants of their own (kOptAnyHit): BVH / parity / full-frame / LDS-poison tests, C4 and C5
mkdir -p gpurun_out
O=gpurun_out
R=r05_17
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_parity.py tests/test_gpu_fullframe.py tests/test_gpu_lds_poison.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config']['launch_mode'], d['config'].get('kernel_option_bits'))"; }
for rep in 1 2; do
timeout -k 10 170 python3 bench.py --config c5 --spp 16 --steps 8 --warmup 5 --no-cpu-baseline > $O/${R}_c5_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5_$rep.json c5
done
timeout -k 10 170 python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline > $O/${R}_c4.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4.json c4
