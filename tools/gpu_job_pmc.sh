# r06 run 49: executed-work counts, PMC traffic and instruction mixes of the final kernels (the sky kernel in one-tile
# blocks): C2, the share-8 step, C4 (iqpt_anyhit_kernel), C5
mkdir -p gpurun_out
O=gpurun_out
R=r06_49
export TMPDIR=/tmp
for c in c2 c4 c5; do
S=""; [ $c = c5 ] && S="--spp 16"; [ $c = c4 ] && S="--spp 16"
timeout -k 10 300 python3 tools/work_counters.py --config $c $S --out $O/work_${c}_r06.json > $O/${R}_work_$c.log 2>&1 || { tail -20 $O/${R}_work_$c.log; exit 1; }
python3 -c "import json; d=json.load(open('$O/work_${c}_r06.json')); print('$c', d['kernel_sha16'], d['per_ray'], d['flops_per_ray'])"
done
pmc() {  # name, counters, bench args
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d $O/${R}_$1 -o run -- $B $3 > $O/${R}_$1.log 2>&1 || { tail -20 $O/${R}_$1.log; exit 1; }
  echo "pmc $1 done"
}
csvf() { find $O/${R}_$1 -name "*counter_collection.csv" | head -1; }
MA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32"
MB="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
B="python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0"
pmc c2_fetch FETCH_SIZE "" && pmc c2_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c2_fetch) $(csvf c2_write) c2 $O/pmc_traffic_c2_r06.json 64 0 iqpt_render_kernel,iqpt_sky_kernel > /dev/null
pmc c2_mixa "$MA" "" && pmc c2_mixb "$MB" ""
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_pmc_mix_r06.json iqpt_render_kernel iqpt_render_kernel > /dev/null
python3 tools/pmc_mix.py $(csvf c2_mixa) $(csvf c2_mixb) c2 1 $O/c2_sky_pmc_mix_r06.json iqpt_sky_kernel iqpt_sky_kernel > /dev/null
pmc s8_mixa "$MA" "--share-of 8" && pmc s8_mixb "$MB" "--share-of 8"
for k in spec fan sky; do
python3 tools/pmc_mix.py $(csvf s8_mixa) $(csvf s8_mixb) c3_share8 1 $O/pmc_mix_${k}_n8_r06.json iqpt_${k}_kernel iqpt_${k}_kernel > /dev/null
done
B="python3 bench.py --config c4 --steps 3 --warmup 5 --no-cpu-baseline --verify-rows 0"
pmc c4_fetch FETCH_SIZE "" && pmc c4_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c4_fetch) $(csvf c4_write) c4 $O/pmc_traffic_c4_256spp_r06.json 256 3 iqpt_anyhit_kernel > /dev/null
pmc c4_mixa "$MA" "" && pmc c4_mixb "$MB" ""
python3 tools/pmc_mix.py $(csvf c4_mixa) $(csvf c4_mixb) c4 1 $O/c4_pmc_mix_r06.json iqpt_anyhit_kernel iqpt_anyhit_kernel > /dev/null
B="python3 bench.py --config c5 --spp 16 --steps 3 --warmup 3 --no-cpu-baseline --verify-rows 0"
pmc c5_fetch FETCH_SIZE "" && pmc c5_write WRITE_SIZE ""
python3 tools/pmc_traffic.py $(csvf c5_fetch) $(csvf c5_write) c5 $O/pmc_traffic_c5_16spp_r06.json 16 3 > /dev/null
pmc c5_mixa "$MA" "" && pmc c5_mixb "$MB" ""
python3 tools/pmc_mix.py $(csvf c5_mixa) $(csvf c5_mixb) c5 1 $O/c5_pmc_mix_r06.json iqpt_render_kernel iqpt_render_kernel > /dev/null
for f in c2_pmc_mix_r06 c2_sky_pmc_mix_r06 pmc_mix_spec_n8_r06 pmc_mix_fan_n8_r06 pmc_mix_sky_n8_r06 c4_pmc_mix_r06 c5_pmc_mix_r06; do
python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['kernel_sha16'], d['kernel_ms_profiled'], d['valu_busy_frac'], d['mean_waves_per_simd'], d['wave_time_split'])"
done
for f in pmc_traffic_c2_r06 pmc_traffic_c4_256spp_r06 pmc_traffic_c5_16spp_r06; do
python3 -c "import json; d=json.load(open('$O/$f.json')); print('$f', d['kernel_sha16'], round(d['hbm_bytes_per_launch'] / 1e6, 1), 'MB')"
done
