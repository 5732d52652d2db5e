# r04 run 30: final-tree spec kernel diagnostics at the N = 8 share — per-block timeline (beside the fan kernel
# and alone) and the PMC instruction mix of the spec / fan / sky kernels
mkdir -p gpurun_out
O=gpurun_out
R=r04_30
timeout -k 10 200 python3 tools/spec_timeline.py --share 8 --specfan 0 --out $O/${R}_timeline_n8_beside.json > $O/${R}_tl0.log 2>&1 || { tail -20 $O/${R}_tl0.log; exit 1; }
tail -8 $O/${R}_tl0.log
timeout -k 10 200 python3 tools/spec_timeline.py --share 8 --specfan 1 --out $O/${R}_timeline_n8_alone.json > $O/${R}_tl1.log 2>&1 || { tail -20 $O/${R}_tl1.log; exit 1; }
tail -8 $O/${R}_tl1.log
export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VALU_TRANS_F32"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $A --kernel-trace --output-format csv -d $O/${R}_mixa -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 --share-of 8 > $O/${R}_mixa.log 2>&1 || { tail -20 $O/${R}_mixa.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc $B --kernel-trace --output-format csv -d $O/${R}_mixb -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --verify-rows 0 --share-of 8 > $O/${R}_mixb.log 2>&1 || { tail -20 $O/${R}_mixb.log; exit 1; }
