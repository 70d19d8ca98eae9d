#!/bin/bash
# Decoded paths on the latency plan: the tree against the same kernel with no path-record stores to
# HBM (-DSVH_PIPE_NOPSTORE, timing only), interleaved, HIP-event time of the pass; the first two
# without the traceback launches (SVH_PIPE_SKIP_TRACEBACK=1), the last the whole pass.  Then per-wave
# stamps of the path variant (diagnostic build).
OUT=${1:-gpurun_out/pstore}
mkdir -p $OUT
export TMPDIR=/tmp
ROUNDS=3 timeout -k 10 400 bash tools/ab_time.sh "--steps 20 --warmup 3 --paths" tree:SVH_PIPE_SKIP_TRACEBACK=1,SVH_LAUNCH_NOCHECK=1 pnostore:SVH_PIPE_SKIP_TRACEBACK=1,SVH_LAUNCH_NOCHECK=1 tree > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 --paths > $OUT/stamps_paths.log 2>&1
grep -h "pipe stamps\|last sweep" $OUT/stamps_paths.log
