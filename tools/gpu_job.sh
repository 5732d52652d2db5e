# r05 run 19: kernel traces of the share-8 step with the gather, block kernel and queue mode (4 blocks per CU)
mkdir -p gpurun_out
O=gpurun_out
R=r05_19
export TMPDIR=/tmp
for q in 0 1; do
Q="--spec-queue 0"; [ $q = 1 ] && Q="--spec-queue 1 --spec-qbpc 4"
timeout -k 10 170 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${R}_kt_s8_q$q -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --share-of 8 --self-gather $Q > $O/${R}_kt_q$q.json 2> $O/${R}_e.err || { tail -20 $O/${R}_e.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/${R}_kt_q$q.json').read().strip().splitlines()[-1]); print('q$q', d['ms_per_step'], d['roofline'].get('kernel_avg_ms'))"
done
