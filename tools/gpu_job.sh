# r06 run 8: measurements keyed on this tree's kernel sources: executed-work counts (C2 / C4 / C5), the default line
# with the -march=native 60-s CPU baseline, rocprofv3 kernel stats + span of the default line and the share-8 step,
# PMC traffic and instruction mix of C2 (render + sky) and of the share-8 step (spec / fan / sky), C5 16-spp traffic
mkdir -p gpurun_out
O=gpurun_out
R=r06_08
export TMPDIR=/tmp
for c in c2 c4 c5; do
S=""; [ $c = c5 ] && S="--spp 16"; [ $c = c4 ] && S="--spp 16"
timeout -k 10 300 python3 tools/work_counters.py --config $c $S --out $O/work_${c}_r06.json > $O/${R}_work_$c.log 2>&1 || { tail -20 $O/${R}_work_$c.log; exit 1; }
tail -c 300 $O/${R}_work_$c.log; echo
done
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], r.get('frac'), c.get('value'), c.get('build'), c.get('cores'), c.get('all_cpus_linear_estimate'))"; }
timeout -k 10 400 python3 bench.py > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_n1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_prof_n1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_n1.json prof_n1
python3 tools/kernel_span.py $(find $O/${R}_prof_n1 -name "run_kernel_trace.csv" | head -1) c2 20 $O/c2_kernel_trace_span_r06.json iqpt_render_kernel,iqpt_sky_kernel
cp $(find $O/${R}_prof_n1 -name "run_kernel_stats.csv" | head -1) $O/c2_kernel_stats_r06.csv
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_s8 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 > $O/${R}_prof_s8.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_s8.json prof_s8
python3 tools/kernel_span.py $(find $O/${R}_prof_s8 -name "run_kernel_trace.csv" | head -1) c3_share8 20 $O/c3_share8_kernel_trace_span_r06.json iqpt_spec_kernel,iqpt_fan_kernel
cp $(find $O/${R}_prof_s8 -name "run_kernel_stats.csv" | head -1) $O/c3_share8_kernel_stats_r06.csv
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0"
pmc() {  # name, counters, bench args
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/${R}_$1 -o run -- $B $3 > $O/${R}_$1.log 2>&1 || { tail -20 $O/${R}_$1.log; exit 1; }
  echo "pmc $1 done"
}
csvf() { find $O/${R}_$1 -name "*counter_collection.csv" | head -1; }
pmc c2_fetch FETCH_SIZE "" && pmc c2_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c2_fetch) $(csvf c2_write) c2 $O/pmc_traffic_c2_r06.json 64 0 iqpt_render_kernel,iqpt_sky_kernel
pmc c2_mixa "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32" "" && pmc c2_mixb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ""
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_pmc_mix_r06.json iqpt_render_kernel iqpt_render_kernel > /dev/null
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_sky_pmc_mix_r06.json iqpt_sky_kernel iqpt_sky_kernel > /dev/null
pmc s8_mixa "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32" "--share-of 8" && pmc s8_mixb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "--share-of 8"
for k in spec fan sky; do
python3 tools/pmc_mix.py $(csvf s8_mixa) $(csvf s8_mixb) c3_share8 1 $O/pmc_mix_${k}_n8_r06.json iqpt_${k}_kernel iqpt_${k}_kernel > /dev/null
done
for f in c2_pmc_mix_r06 c2_sky_pmc_mix_r06 pmc_mix_spec_n8_r06 pmc_mix_fan_n8_r06 pmc_mix_sky_n8_r06; do
python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['kernel_sha16'], d['kernel_ms_profiled'], d['valu_busy_frac'], d['wave_time_split'])"
done
B="python3 bench.py --config c5 --spp 16 --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0"
pmc c5_fetch FETCH_SIZE "" && pmc c5_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c5_fetch) $(csvf c5_write) c5 $O/pmc_traffic_c5_16spp_r06.json 16 3
