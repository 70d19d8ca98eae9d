#!/bin/bash
# Prologue: the pair tables' compiler barrier after the prologue's other loads (SVH_PIPE_LATEOPQ,
# tree) against right after the table loads (lateopq0): latency-plan GPU tests, interleaved A/B,
# per-row stamps of the tree.
OUT=${1:-gpurun_out/lateopq}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipe_gpu.py tests/test_reference_scope_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ROUNDS=4 timeout -k 10 500 bash tools/ab_time.sh "--steps 20 --warmup 3" tree lateopq0 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 2 --warmup 1 > $OUT/stamps_tree.log 2>&1
grep -h -E "^  seq 0:" $OUT/stamps_tree.log | cut -c1-200
