#!/bin/bash
# Round 4 GPU session 11: count publish by every lane (SVH_PIPE_PUT=1, put1) against the tree.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s11}
mkdir -p $OUT
ROUNDS=5 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree put1 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
