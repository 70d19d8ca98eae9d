#!/bin/bash
# Where the decoded-path pass's forward kernel spends its time over the scores kernel: the tree, no
# HBM record stores (pnostore), no fold of the record ring (nofold), no record ring at all (nopring),
# all without the traceback launches (SVH_PIPE_SKIP_TRACEBACK=1, timing only), and the scores pass.
OUT=${1:-gpurun_out/psplit}
mkdir -p $OUT
export TMPDIR=/tmp
E=SVH_PIPE_SKIP_TRACEBACK=1,SVH_LAUNCH_NOCHECK=1
ROUNDS=3 timeout -k 10 600 bash tools/ab_time.sh "--steps 20 --warmup 3 --paths" tree:$E pnostore:$E nofold:$E nopring:$E > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
