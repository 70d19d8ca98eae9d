#!/bin/bash
# Round 4 GPU session 12: exchange groups of 16 observations (g16: pipe_kernel_g16.h, A/B build
# only) on the latency-plan parity tests, then interleaved timing against the tree.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s12}
mkdir -p $OUT
SVH_LIB=build_ab/g16/libspec_viterbi_hip.so timeout -k 10 300 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread -k "(headline or table_modes or long_sequence or covid_ragged or test_pipe_sequence_lengths) and not paths" > $OUT/pytest_g16.log 2>&1; rc=$?
tail -3 $OUT/pytest_g16.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=5 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree g16 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
