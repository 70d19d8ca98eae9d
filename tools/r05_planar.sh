#!/bin/bash
# Planar path-record ring: the GPU tests of the latency plan and every decoded-path test, then the
# path pass's time (whole pass and forward kernels only) for comparison with the records before
# (profiles/r05_paths/ab_split.log: forward 0.364-0.372 ms, whole pass ~0.39).
OUT=${1:-gpurun_out/planar}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_pipe_gpu.py tests/test_reference_scope_gpu.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
E=SVH_PIPE_SKIP_TRACEBACK=1,SVH_LAUNCH_NOCHECK=1
ROUNDS=3 timeout -k 10 400 bash tools/ab_time.sh "--steps 20 --warmup 3 --paths" tree tree:$E > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
