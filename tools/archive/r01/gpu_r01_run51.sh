# round-1 GPU run 51: per-wave timeline of the C2 launch (kOptStats variant), 64 and 256 spp
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spp in 64 256; do
timeout -k 10 200 python3 tools/ab_kernel.py --config c2 --spp $spp --rounds 3 --variants "default=2863" --out gpurun_out/ab51_$spp.json > gpurun_out/ab51_$spp.log 2>&1 || { echo FAILED; tail -20 gpurun_out/ab51_$spp.log; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab51_$spp.json')); print($spp, d['variants']['default']['median_ms'], json.dumps(d['wave_timeline']))"
done
echo DONE
