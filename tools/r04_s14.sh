#!/bin/bash
# Round 4 GPU session 14: G16 count-read placement (step 4, 8 = g16, 12 of the group; then 12, 14, 15) against the tree.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s14}
mkdir -p $OUT
ROUNDS=6 timeout -k 10 500 bash tools/ab_time.sh "--steps 30 --warmup 3" tree g16c12 g16c14 g16c15 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
