# round-2 run 37: chain-kernel timing ablations (A/B library, NOT exact): all-tiles chain at N = 1, split-set chain at N = 8
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 64 128 256 512 960; do
  timeout -k 10 200 python3 tools/split_share.py --ab --diag $d --modes chain --chain-waves 16a --ns 1,8 --launches 5 --warm 1 > gpurun_out/r02_run37_d$d.log 2>&1 || exit 1
done
