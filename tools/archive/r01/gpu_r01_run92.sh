# round-1 GPU run 92: C5 bench at 40 timed steps, two processes (run 91's 10-step C5 line was 5 % below v10)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for p in 1 2; do
timeout -k 10 400 python3 bench.py --config c5 --spp 1 --steps 40 --warmup 5 --no-cpu-baseline --pmc-json profiles/r01_pmc_traffic_c5_v4.json --pmc-mix-json profiles/r01_c5_pmc_mix_v3.json > gpurun_out/b92_c5_$p.json 2> gpurun_out/b92_c5_$p.err || { echo BENCH5_FAILED; tail -20 gpurun_out/b92_c5_$p.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b92_c5_$p.json'));print($p, d['value'], d['roofline']['kernel_avg_ms'], d['bitexact_frac_vs_oracle'])"
done
echo DONE
