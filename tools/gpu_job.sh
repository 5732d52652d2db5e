# r05 run 36: whole-wave refills by default for streamed scenes (K = 64), the refill size a runtime value for
# resident plain launches too (default 1): tests, the C2 line at resident K = 1 / 16 / 64 x2 alternated, the C5
# and C4 lines, executed-work counts on these kernel sources, C5 traffic
mkdir -p gpurun_out
O=gpurun_out
R=r05_36
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_bvh.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
for rep in 1 2; do
for k in 1 16 64; do
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --resident-refill $k > $O/${R}_c2_k${k}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c2_k${k}_$rep.json c2_k${k}_$rep
done
done
timeout -k 10 240 python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline > $O/${R}_c5.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5.json c5
timeout -k 10 240 python3 bench.py --config c4 --steps 3 --no-cpu-baseline > $O/${R}_c4.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4.json c4
for c in c2 c4 c5; do
S=""; [ $c = c5 ] && S="--spp 16"; [ $c = c4 ] && S="--spp 16"
timeout -k 10 300 python3 tools/work_counters.py --config $c $S --out $O/work_${c}_r05.json > $O/${R}_work_$c.log 2>&1 || { tail -20 $O/${R}_work_$c.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/work_${c}_r05.json')); print('work $c', d['kernel_sha16'], d['rays'], d['flops_per_ray'])"
done
csvf() { find $O/${R}_$1 -name "*counter_collection.csv" | head -1; }
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${R}_c5_$c -o run -- python3 bench.py --config c5 --spp 16 --steps 3 --no-cpu-baseline --verify-rows 0 > $O/${R}_c5_$c.log 2>&1 || { tail -20 $O/${R}_c5_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $(csvf c5_FETCH_SIZE) $(csvf c5_WRITE_SIZE) c5 $O/pmc_traffic_c5_16spp_r05.json 16 3 > /dev/null
python3 -c "import json; d=json.load(open('$O/pmc_traffic_c5_16spp_r05.json')); print('traffic c5', d['fetch_bytes_corrected']/1e9, d['write_bytes']/1e9, d['hbm_bytes_per_launch']/1e9)"
