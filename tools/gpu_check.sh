#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, then the rocprofv3 evidence.
# Every GPU step has its own time limit; steps are chained with && so the first failure ends it.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r03}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_${TAG}.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 &&
TAG=$TAG bash tools/profile.sh
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log; tail -2 gpurun_out/bench_${TAG}.log
exit $rc
