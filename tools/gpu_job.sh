# r05 run 31: streamed-scene waves take new pixels 16 idle lanes at a time by default (p.refill_min for STREAM
# variants, iqpt_debug_set_stream_refill): BVH / full-frame tests (refill 1 / 16 / 64 against the oracle), the
# C5 and C4 lines at refill 1 / 16 / 32 alternated, executed-work counts on these kernel sources, C5 / C4 traffic
mkdir -p gpurun_out
O=gpurun_out
R=r05_31
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('stream_refill'))"; }
for rep in 1 2; do
for k in 1 16 32; do
timeout -k 10 240 python3 bench.py --config c5 --spp 16 --steps 10 --warmup 3 --no-cpu-baseline --stream-refill $k > $O/${R}_c5_k${k}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5_k${k}_$rep.json c5_k${k}_$rep
done
done
for k in 1 16 32; do
timeout -k 10 240 python3 bench.py --config c4 --steps 3 --warmup 3 --no-cpu-baseline --stream-refill $k > $O/${R}_c4_k${k}.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c4_k${k}.json c4_k${k}
done
for c in c2 c4 c5; do
S=""; [ $c = c5 ] && S="--spp 16"; [ $c = c4 ] && S="--spp 16"
timeout -k 10 300 python3 tools/work_counters.py --config $c $S --out $O/work_${c}_r05.json > $O/${R}_work_$c.log 2>&1 || { tail -20 $O/${R}_work_$c.log; exit 1; }
tail -c 300 $O/${R}_work_$c.log; echo
done
csvf() { find $O/${R}_$1 -name "*counter_collection.csv" | head -1; }
pmc() {  # name, counter, bench args
  timeout -s KILL 200 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/${R}_$1 -o run -- python3 bench.py --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0 $3 > $O/${R}_$1.log 2>&1 || { tail -20 $O/${R}_$1.log; exit 1; }
}
pmc c5_fetch FETCH_SIZE "--config c5 --spp 16" && pmc c5_write WRITE_SIZE "--config c5 --spp 16"
python3 tools/pmc_traffic.py $(csvf c5_fetch) $(csvf c5_write) c5 $O/pmc_traffic_c5_16spp_r05.json 16 3 > /dev/null
pmc c4_fetch FETCH_SIZE "--config c4" && pmc c4_write WRITE_SIZE "--config c4"
python3 tools/pmc_traffic.py $(csvf c4_fetch) $(csvf c4_write) c4 $O/pmc_traffic_c4_256spp_r05.json 256 3 > /dev/null
for c in c5_16spp c4_256spp; do
python3 -c "import json; d=json.load(open('$O/pmc_traffic_${c}_r05.json')); print('traffic $c', d['fetch_bytes_corrected']/1e9, d['write_bytes']/1e9, d['hbm_bytes_per_launch']/1e9)"
done
