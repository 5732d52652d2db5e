# round-1 GPU run 11: multi-rank rehearsal (2 ranks, gloo, one GPU) vs N=1 frame bit-equality;
# bench of the current kernel with cpu_baseline; rocprof stats; PMC traffic passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify-rows 4 --save-frame gpurun_out/frame_n1.npy > gpurun_out/r11_n1.json 2> gpurun_out/r11_n1.err || { echo N1_FAILED; tail -30 gpurun_out/r11_n1.err; exit 1; }
cat gpurun_out/r11_n1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --one-device --steps 2 --warmup 1 --verify-rows 4 --save-frame gpurun_out/frame_n2.npy > gpurun_out/r11_n2.json 2> gpurun_out/r11_n2.err || { echo N2_FAILED; tail -30 gpurun_out/r11_n2.err; exit 1; }
cat gpurun_out/r11_n2.json
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/frame_n1.npy"); b = np.load("gpurun_out/frame_n2.npy")
print("frames", a.shape, b.shape, "bit-equal:", bool(np.array_equal(a.view(np.uint32), b.view(np.uint32))))
PY
timeout -k 10 400 python bench.py > gpurun_out/r11_bench.json 2> gpurun_out/r11_bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/r11_bench.err; exit 1; }
cat gpurun_out/r11_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r11_prof.json 2> gpurun_out/r11_prof.err || { echo PROF_FAILED; tail -20 gpurun_out/r11_prof.err; exit 1; }
cat gpurun_out/r11_prof.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc11_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc11_fetch.log 2>&1 || { echo PMC1_FAILED; tail -20 gpurun_out/pmc11_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc11_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --verify-rows 0 > gpurun_out/pmc11_write.log 2>&1 || { echo PMC2_FAILED; tail -20 gpurun_out/pmc11_write.log; exit 1; }
find gpurun_out/prof11 gpurun_out/pmc11_fetch gpurun_out/pmc11_write -name "*.csv"
echo DONE
