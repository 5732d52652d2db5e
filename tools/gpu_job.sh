# r06 run 24: the two-ray kernel's shading rounds as a loop (-DIQPT_PIPE_ROUNDS_LOOP=1: 24 % less code) against the
# unrolled rounds, the default line alternated x3
mkdir -p gpurun_out
O=gpurun_out
R=r06_24
export TMPDIR=/tmp
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], d['config'].get('kernel_option_bits'))"; }
for i in 1 2 3; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/${R}_base_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_base_$i.json base$i
timeout -k 10 200 python3 bench.py --no-cpu-baseline --lib path-tracer-and-rasterizer-engine_amd/build/abr6/libiqpt_rl.so > $O/${R}_rl_$i.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_rl_$i.json rl$i
done
