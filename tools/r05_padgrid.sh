#!/bin/bash
# Padded grid (every XCD class holds the same number of workgroups; leftover rows class-ordered) and
# the early next-vector read (SVH_PIPE_EARLYV) and the exchange helpers (SVH_PIPE_XHELP): latency-plan
# GPU tests, interleaved A/B against the previous commit (prev) and the tree without the helpers
# (xhelp0), per-row stamps.
OUT=${1:-gpurun_out/padgrid}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipe_gpu.py tests/test_reference_scope_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ROUNDS=4 timeout -k 10 500 bash tools/ab_time.sh "--steps 20 --warmup 3" tree prev xhelp0 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tree.log 2>&1
grep -h "pipe stamps" $OUT/stamps_tree.log
