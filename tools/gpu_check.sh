#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, then the rocprofv3 evidence.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
bash tools/profile.sh
rc=$?
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/bench.log
exit $rc
