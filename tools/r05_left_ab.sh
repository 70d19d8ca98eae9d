#!/bin/bash
# Remaining rows of the XCD-class mapping from one start-order ticket counter (tree) against the
# class-ordered spare slots of the previous commit (prev): latency-plan GPU tests (two 50-row
# batches at once on two streams among them), interleaved A/B.
OUT=${1:-gpurun_out/left}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipe_gpu.py tests/test_reference_scope_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ROUNDS=4 timeout -k 10 500 bash tools/ab_time.sh "--steps 20 --warmup 3" tree prev > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
