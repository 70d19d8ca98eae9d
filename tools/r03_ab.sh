#!/bin/bash
# A/B of library variants on the headline workload, then wall-clock wave stamps of diagnostic
# builds (-DSVH_PIPE_DIAG).
#   STAMPS="rt rt0" tools/r03_ab.sh OUTDIR VARIANT...   (VARIANT = name under build_ab, or "tree")
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_pipe_gpu.py -q -m gpu --maxfail=3 --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; case $rc in 0) ;; *) exit $rc;; esac
ROUNDS=${ROUNDS:-3} bash tools/ab_time.sh "--steps 30 --warmup 3" "$@" > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in $STAMPS; do
    SVH_LIB=build_ab/$v/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_$v.log 2>&1 || exit $?
    grep "pipe wall" $OUT/stamps_$v.log | tail -1
done
