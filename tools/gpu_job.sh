# r05 run 24: slot colours with non-temporal stores (build/ab/libiqpt_ntres.so) against this tree, share 8 / 4
# alternated x3 (bench's band check vs the oracle in every line), and the spec-kernel gaps in a kernel trace
mkdir -p gpurun_out
O=gpurun_out
R=r05_24
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'])"; }
AB=path-tracer-and-rasterizer-engine_amd/build/ab
for rep in 1 2 3; do
for n in 8 4; do
for lib in new nt; do
L=""; [ $lib = nt ] && L="--lib $AB/libiqpt_ntres.so"
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of $n --self-gather $L > $O/${R}_s${n}g_${lib}_$rep.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${n}g_${lib}_$rep.json share${n}_$lib
done
done
done
timeout -k 10 170 rocprofv3 --kernel-trace --output-format csv -d $O/${R}_kt_nt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather --lib $AB/libiqpt_ntres.so > $O/${R}_kt_nt.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
python3 - <<PY
import csv
rows = list(csv.DictReader(open('$O/${R}_kt_nt/run_kernel_trace.csv')))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows if 'iqpt_spec_kernel' in r['Kernel_Name'])[-21:]
gaps = sorted((ks[i+1][0] - ks[i][1]) / 1000 for i in range(len(ks) - 1))
d = sorted((e - s) / 1000 for s, e in ks)
print('nt: spec gaps median', gaps[len(gaps)//2], 'min', gaps[0], 'max', gaps[-1], 'dur median', d[len(d)//2], 'period', round((ks[-1][1] - ks[0][1]) / 20 / 1000, 1))
PY
