# round-2 run 31: overlap A/B (tile order, slots left per CU) on the default C2 bench, 40 steps each
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 40 --no-cpu-baseline --verify-rows 0"
for v in off s1 r1 off2 s1b; do
  case $v in
    off|off2) E=""; A="--overlap off";;
    s1|s1b) E="IQPT_OVL_READY=0 IQPT_OVL_FREE=1"; A="";;
    s2) E="IQPT_OVL_READY=0 IQPT_OVL_FREE=2"; A="";;
    s0) E="IQPT_OVL_READY=0 IQPT_OVL_FREE=0"; A="";;
    r1) E="IQPT_OVL_READY=1 IQPT_OVL_FREE=1"; A="";;
  esac
  env $E timeout -k 10 120 $B $A > gpurun_out/r02_run31_$v.json 2> gpurun_out/r02_run31_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('gpurun_out/r02_run31_$v.json'));print(d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['launch_duration_ms'])")" >> gpurun_out/r02_run31.txt
done
