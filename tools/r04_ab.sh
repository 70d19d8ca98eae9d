#!/bin/bash
# Round 4 A/B on the headline workload: interleaved HIP-event timing of library variants
# (golden-checked), then the no-exchange step time of diagnostic builds (SVH_PIPE_DEBUG=3: every
# exchange off, wrong results by design) from the wave wall-clock stamps.
#   STAMPS="t0d t4d" tools/r04_ab.sh OUTDIR VARIANT...   (VARIANT = name under build_ab, or "tree")
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
ROUNDS=${ROUNDS:-3} bash tools/ab_time.sh "--steps 30 --warmup 3" "$@" > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in $STAMPS; do
    for d in 1 3; do
        SVH_LIB=build_ab/$v/libspec_viterbi_hip.so SVH_PIPE_DEBUG=$d timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_${v}_$d.log 2>&1 || exit $?
        echo "$v debug=$d: $(grep 'pipe wall' $OUT/stamps_${v}_$d.log | tail -1) | $(grep 'pipe stamps' $OUT/stamps_${v}_$d.log | tail -1)"
    done
done
