#!/bin/bash
# Slow path with one LDS round trip (SVH_PIPE_SLOW1, tree) against two (slow10):
# latency-plan GPU tests, interleaved A/B, per-row stamps of the tree.
OUT=${1:-gpurun_out/slow1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipe_gpu.py tests/test_reference_scope_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ROUNDS=4 timeout -k 10 500 bash tools/ab_time.sh "--steps 20 --warmup 3" tree slow10 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 2 --warmup 1 > $OUT/stamps_tree.log 2>&1
grep -h -A 21 "wait split by role" $OUT/stamps_tree.log
