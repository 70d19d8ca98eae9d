#!/bin/bash
# Cross-XCD granule prefetch depth: the tree (4 groups for consumers whose producer is on another
# XCD) against depth 2 everywhere (gx2); stamps of both (diagnostic builds).
OUT=${1:-gpurun_out/gpfx}
mkdir -p $OUT
export TMPDIR=/tmp
ROUNDS=3 timeout -k 10 400 bash tools/ab_time.sh "--steps 20 --warmup 3" tree gx2 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in diag diaggx2; do
  SVH_LIB=build_ab/$v/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_$v.log 2>&1
  grep -h "pipe stamps\|last sweep\|seq 48\|seq 49\|seq 0:\|seq 12:" $OUT/stamps_$v.log | cut -c1-260
done
