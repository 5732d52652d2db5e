# round-2 run 43: C2 default bench vs the short pitch-only camera (kOptCamAxis) now that launches overlap, alternating
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 40 --no-cpu-baseline --verify-rows 4"
for r in 1 2 3; do
  timeout -k 10 120 $B > gpurun_out/r02_run43_def_$r.json 2>/dev/null || exit 1
  timeout -k 10 120 $B --kernel-options 0x44b2f > gpurun_out/r02_run43_cam_$r.json 2>/dev/null || exit 1
done
