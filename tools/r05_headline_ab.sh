#!/bin/bash
# Headline kernel, where the exchange costs: the tree, the tree with every neighbour wait removed
# (-DSVH_PIPE_NOWAIT: exchange work done, never held up; wrong results), and no exchange at all
# (-DSVH_PIPE_DIAG build with SVH_PIPE_DEBUG=3; wrong results).  Interleaved rounds, HIP-event time.
OUT=${1:-gpurun_out/headline_ab}
mkdir -p $OUT
export TMPDIR=/tmp
ROUNDS=3 timeout -k 10 500 bash tools/ab_time.sh "--steps 20 --warmup 3" tree nowait diag:SVH_PIPE_DEBUG=3 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tree.log 2>&1
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=3 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_noexch.log 2>&1
grep -h "pipe stamps" $OUT/stamps_*.log
# decoded paths: the tree's PATHS pass against the same pass without the per-step LDS record store
ROUNDS=3 timeout -k 10 300 bash tools/ab_time.sh "--steps 20 --warmup 3 --paths" tree nopring > $OUT/ab_paths.log 2>&1 || { cat $OUT/ab_paths.log; exit 1; }
cat $OUT/ab_paths.log
