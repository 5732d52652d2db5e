# r05 run 37: final tree (kernel_sha16 d641492d1326f709, whole-wave refills for streamed scenes): pytest -m gpu,
# smoke, the driver's default command, rocprofv3 kernel stats / trace span of the default line and of the C5 line,
# the share-8 step with the gather
mkdir -p gpurun_out
O=gpurun_out
R=r05_37
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/${R}_tests.log 2>&1 || { tail -40 $O/${R}_tests.log; exit 1; }
tail -1 $O/${R}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/${R}_smoke.log 2>&1 || { tail -20 $O/${R}_smoke.log; exit 1; }
tail -1 $O/${R}_smoke.log
pr() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']; c=d.get('cpu_baseline') or {}; print('$2', d['value'], d['ms_per_step'], r.get('kernel_avg_ms'), d['bitexact_frac_vs_oracle'], r.get('frac'), c.get('value'))"; }
timeout -k 10 300 python3 bench.py > $O/${R}_default.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_default.json default
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_n1 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/${R}_prof_n1.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_n1.json prof_n1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_prof_c5 -o run -- python3 bench.py --config c5 --spp 16 --steps 10 --no-cpu-baseline > $O/${R}_prof_c5.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_prof_c5.json prof_c5
python3 - <<'EOF'
import csv, glob, json
for tag, n in (("n1", 20), ("c5", 10)):
    f = glob.glob(f"gpurun_out/r05_37_prof_{tag}/**/run_kernel_trace.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "iqpt_render_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    last = rows[-n:]
    span = (max(int(r["End_Timestamp"]) for r in last) - int(last[0]["Start_Timestamp"])) / n / 1e6
    own = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / n / 1e6
    print(tag, "launches", len(rows), "span per launch ms", round(span, 4), "own duration ms", round(own, 4), f)
EOF
timeout -k 10 170 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather > $O/${R}_s8g.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
pr $O/${R}_s8g.json share8_gather
