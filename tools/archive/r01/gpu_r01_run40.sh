# round-1 GPU run 40: 2-rank rehearsals of both bench modes on one GPU (after the BVH and mean-term changes)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 10 > gpurun_out/r40_strong1.json 2> gpurun_out/r40_strong1.err || { echo BENCH2_FAILED; tail -30 gpurun_out/r40_strong1.err; exit 1; }
cat gpurun_out/r40_strong1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --backend gloo --one-device --steps 2 --warmup 1 --verify-rows 4 --save-frame gpurun_out/frame40_weak2.npy > gpurun_out/r40_weak2.json 2> gpurun_out/r40_weak2.err || { echo WEAK2_FAILED; tail -30 gpurun_out/r40_weak2.err; exit 1; }
cat gpurun_out/r40_weak2.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 bench.py --gpus 2 --backend gloo --one-device --scaling strong --steps 2 --warmup 1 --verify-rows 4 --save-frame gpurun_out/frame40_strong2.npy > gpurun_out/r40_strong2.json 2> gpurun_out/r40_strong2.err || { echo STRONG2_FAILED; tail -30 gpurun_out/r40_strong2.err; exit 1; }
cat gpurun_out/r40_strong2.json
timeout -k 10 300 python bench.py --scaling strong --no-cpu-baseline --steps 2 --warmup 1 --verify-rows 4 --save-frame gpurun_out/frame40_strong1.npy > /dev/null 2>&1 || { echo SAVE1_FAILED; exit 1; }
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/frame40_strong1.npy"); b = np.load("gpurun_out/frame40_strong2.npy")
print("strong: 2-rank frame bit-equal to 1-rank:", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))))
w = np.load("gpurun_out/frame40_weak2.npy")
print("weak: mean frame shape", w.shape, "finite", bool(np.isfinite(w[:, :3]).all()))
PY
echo DONE
