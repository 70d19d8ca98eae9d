#!/bin/bash
# Round 4 GPU session 4: why the pair-table step (TM=1) is slower in the pipeline than TM=0.
# Diagnostic build t1d (-DSVH_PIPE_DIAG): wave timeline (SVH_PIPE_DEBUG=1) and the no-exchange
# step (SVH_PIPE_DEBUG=3) for TM 1 / 0 / 2; A/B of the batched LDS ring (r8) in both modes;
# strong-scaling shares.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s4}
mkdir -p $OUT
for tm in 1 0 2; do
    for d in 1 3; do
        SVH_PIPE_TM=$tm SVH_LIB=build_ab/t1d/libspec_viterbi_hip.so SVH_PIPE_DEBUG=$d timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tm${tm}_$d.log 2>&1 || { tail $OUT/stamps_tm${tm}_$d.log; exit 1; }
        echo "tm$tm debug=$d: $(grep 'pipe wall' $OUT/stamps_tm${tm}_$d.log | tail -1) | $(grep 'pipe stamps' $OUT/stamps_tm${tm}_$d.log | tail -1)"
    done
done
ROUNDS=3 timeout -k 10 300 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_TM=0 r8 r8:SVH_PIPE_TM=0 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for sh in covid emit50; do
    timeout -k 10 120 python3 tools/shard_shares.py --shard $sh > $OUT/shares_$sh.json 2> $OUT/shares_$sh.err || { cat $OUT/shares_$sh.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/shares_$sh.json'));print('$sh', {k:(v['makespan_ms'],v['forecast_speedup']) for k,v in d['ranks'].items()})"
done
