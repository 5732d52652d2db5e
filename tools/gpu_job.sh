# r05 run 21 (final tree, part 2): executed-work counts of C2 / C4 / C5 on these kernel sources, PMC traffic and
# instruction mixes: C2 at N = 1 (render + sky), the N = 8 share (spec / fan / sky), C5 at 16 spp, C4 at 256 spp
mkdir -p gpurun_out
O=gpurun_out
R=r05_21
export TMPDIR=/tmp
for c in c2 c4 c5; do
S=""; [ $c = c5 ] && S="--spp 16"; [ $c = c4 ] && S="--spp 16"
timeout -k 10 300 python3 tools/work_counters.py --config $c $S --out $O/work_${c}_r05.json > $O/${R}_work_$c.log 2>&1 || { tail -20 $O/${R}_work_$c.log; exit 1; }
tail -c 400 $O/${R}_work_$c.log; echo
done
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0"
pmc() {  # name, counters, bench args
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/${R}_$1 -o run -- $B $3 > $O/${R}_$1.log 2>&1 || { tail -20 $O/${R}_$1.log; exit 1; }
  echo "pmc $1 done"
}
csvf() { find $O/${R}_$1 -name "*counter_collection.csv" | head -1; }
pmc c2_fetch FETCH_SIZE "" && pmc c2_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c2_fetch) $(csvf c2_write) c2 $O/pmc_traffic_c2_r05.json 64 0 iqpt_render_kernel,iqpt_sky_kernel
pmc c2_mixa "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32" "" && pmc c2_mixb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ""
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_pmc_mix_r05.json iqpt_render_kernel iqpt_render_kernel > /dev/null
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_sky_pmc_mix_r05.json iqpt_sky_kernel iqpt_sky_kernel > /dev/null
python3 -c "import json; [print(k, {x: d[x] for x in ('kernel_ms_profiled','valu_busy_frac','wave_time_split')}) for k, d in ((k, json.load(open('$O/'+k))) for k in ('c2_pmc_mix_r05.json','c2_sky_pmc_mix_r05.json'))]"
pmc s8_mixa "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32" "--share-of 8" && pmc s8_mixb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "--share-of 8"
for k in spec fan sky; do
python3 tools/pmc_mix.py $(csvf s8_mixa) $(csvf s8_mixb) c3_share8 1 $O/pmc_mix_${k}_n8_r05.json iqpt_${k}_kernel iqpt_${k}_kernel > /dev/null
python3 -c "import json; d=json.load(open('$O/pmc_mix_${k}_n8_r05.json')); print('$k', d['kernel_ms_profiled'], d['valu_busy_frac'], d['counters']['SQ_INSTS_VALU'])"
done
B="python3 bench.py --config c5 --spp 16 --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0"
pmc c5_fetch FETCH_SIZE "" && pmc c5_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c5_fetch) $(csvf c5_write) c5 $O/pmc_traffic_c5_16spp_r05.json 16 3
pmc c5_mixa "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32" "" && pmc c5_mixb "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" ""
python3 tools/pmc_mix.py $(csvf c5_mixa) $(csvf c5_mixb) c5 1 $O/c5_pmc_mix_r05.json iqpt_render_kernel iqpt_render_kernel > /dev/null
python3 -c "import json; d=json.load(open('$O/c5_pmc_mix_r05.json')); print('c5 mix', d['kernel_ms_profiled'], d['valu_busy_frac'], d['wave_time_split'])"
B="python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 0"
pmc c4_fetch FETCH_SIZE "" && pmc c4_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c4_fetch) $(csvf c4_write) c4 $O/pmc_traffic_c4_256spp_r05.json 256 3
