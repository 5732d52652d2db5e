# round-1 GPU run 74: compiler scheduling strategies (separate libraries, alternating processes), C2 and C5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
L=path-tracer-and-rasterizer-engine_amd/iqpt
for pass in 1 2; do
  for v in base maxilp memclause; do
    lib=$L/libiqpt_ab_$v.so; [ $v = base ] && lib=$L/libiqpt_ab.so
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c2 --rounds 3 --variants "prod=2863" --out gpurun_out/ab74_c2_${v}_$pass.json > gpurun_out/ab74_c2_${v}_$pass.log 2>&1 || { echo AB_FAILED $v; tail -20 gpurun_out/ab74_c2_${v}_$pass.log; exit 1; }
    timeout -k 10 300 python3 tools/ab_kernel.py --lib $lib --config c5 --spp 1 --rounds 3 --variants "prod=6959" --out gpurun_out/ab74_c5_${v}_$pass.json > gpurun_out/ab74_c5_${v}_$pass.log 2>&1 || { echo AB5_FAILED $v; tail -20 gpurun_out/ab74_c5_${v}_$pass.log; exit 1; }
    python3 -c "
import json
for c in ('c2','c5'):
    d=json.load(open('gpurun_out/ab74_%s_${v}_$pass.json'%c))
    for k,x in d['variants'].items(): print(c, '$v', $pass, x['median_ms'], x['bitexact'])"
  done
done
echo DONE
