set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import sys; sys.path.insert(0,'path-tracer-and-rasterizer-engine_amd'); from iqpt import _build; _build.build_lib(ab=True)"
for sc in empty walls cornell; do
  timeout -k 10 300 python tools/ab_kernel.py --config c2 --scene $sc --rounds 5 --variants "default=39,nopair=35" --out gpurun_out/ab7_$sc.json > gpurun_out/ab7_$sc.log 2>&1 || { echo AB_FAILED $sc; tail -30 gpurun_out/ab7_$sc.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d gpurun_out/pmc7_$sc -o run -- python3 tools/ab_kernel.py --config c2 --scene $sc --only 35 --frames 1 > gpurun_out/pmc7_$sc.log 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/pmc7_$sc.log; exit 1; }
done
python - <<'PY'
import json, csv, collections
for n in ("empty","walls","cornell"):
    d=json.load(open(f"gpurun_out/ab7_{n}.json"))
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(f"gpurun_out/pmc7_{n}/run_counter_collection.csv")):
        if "render_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
    st = d["stats_default"]
    it = st["iterations"]
    print(n, {k:(v["median_ms"], v["bitexact"]) for k,v in d["variants"].items()}, "iters", it, "rays", st["rays"],
          "VALU/iter %.0f SALU/iter %.0f LDS/iter %.1f BR/iter %.1f" % (agg["SQ_INSTS_VALU"]/it, agg["SQ_INSTS_SALU"]/it, agg["SQ_INSTS_LDS"]/it, agg["SQ_INSTS_BRANCH"]/it))
PY
