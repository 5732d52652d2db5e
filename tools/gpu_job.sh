# r06 run 48: the tree's final kernels (the sky kernel in one-tile blocks, run 47): the whole -m gpu suite, smoke, the
# default line with the CPU baseline, rocprofv3 kernel stats + span of the default line (K = 100), the share-8 step,
# C4 and C5, share steps with the gather (executed-work counts and PMC passes: tools/gpu_job_pmc.sh, run 49)
mkdir -p gpurun_out
O=gpurun_out
R=r06_48
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], r.get('frac'), d['config'].get('launch_mode'), c.get('value'), c.get('cores'))"; }
timeout -k 10 400 python3 bench.py > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
prof() {  # tag, config, launches, kernels, bench args
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_$1 -o run -- python3 bench.py --no-cpu-baseline $5 > $O/${R}_prof_$1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
  pr $O/${R}_prof_$1.json prof_$1
  python3 tools/kernel_span.py $(find $O/${R}_prof_$1 -name "run_kernel_trace.csv" | head -1) $2 $3 $O/$2_kernel_trace_span_r06.json $4 > /dev/null
  cp $(find $O/${R}_prof_$1 -name "run_kernel_stats.csv" | head -1) $O/$2_kernel_stats_r06.csv
  python3 -c "import json; d=json.load(open('$O/$2_kernel_trace_span_r06.json')); print('$2', d['kernel_sha16'], d['kernels'])"
}
prof n1 c2 100 iqpt_render_kernel,iqpt_sky_kernel "--steps 100 --warmup 10"
prof s8 c3_share8 100 iqpt_spec_kernel,iqpt_fan_kernel "--steps 100 --warmup 10 --share-of 8"
prof c4 c4 10 iqpt_anyhit_kernel "--config c4 --steps 10"
prof c5 c5 10 iqpt_render_kernel "--config c5 --spp 16 --steps 10"
timeout -k 10 200 python3 bench.py --config c5 --spp 1 --steps 10 --no-cpu-baseline > $O/${R}_c5s1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_c5s1.json c5_spp1
for s in 8 4 2; do
timeout -k 10 200 python3 bench.py --no-cpu-baseline --share-of $s --self-gather > $O/${R}_s${s}.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s${s}.json share${s}_gather
done
