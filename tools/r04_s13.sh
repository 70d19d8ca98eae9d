#!/bin/bash
# Round 4 GPU session 13: G16 count-read placement (step 4, 8 = g16, 12 of the group; then 12, 14, 15) against the tree.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s13}
mkdir -p $OUT
ROUNDS=6 timeout -k 10 500 bash tools/ab_time.sh "--steps 30 --warmup 3" tree g16 g16c4 g16c12 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
