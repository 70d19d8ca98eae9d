#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, then the rocprofv3 evidence.
# Every GPU step has its own time limit.  Test failures do not stop the bench, but a time limit,
# abort or crash (exit 124, 134, 137, 139) ends the call there.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r03}
TESTS=${TESTS:-tests}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $TESTS -v -m gpu --maxfail=20 --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_${TAG}.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_gpu_${TAG}.log
case $rc in 124|134|137|139) echo "pytest ended with $rc: stopping"; exit $rc;; esac
timeout -k 10 300 python bench.py > gpurun_out/bench_${TAG}.log 2>&1 || exit $?
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-400
if [ -z "$NO_PROFILE" ]; then TAG=$TAG bash tools/profile.sh || exit $?; fi
exit $rc
