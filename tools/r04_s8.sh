#!/bin/bash
# Round 4 GPU session 8: GPU suite on the tree (TM 4, chunked result read), host-to-host split,
# every BASELINE config re-measured (profiles/r04_configs), rocprofv3 kernel stats + PMC traffic.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s8}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
cat $OUT/e2e_split.json
OUT=gpurun_out/r04_configs timeout -k 10 900 bash tools/configs.sh > $OUT/configs.log 2>&1 || { tail -30 $OUT/configs.log; exit 1; }
cat $OUT/configs.log | cut -c1-600
TAG=r04_s8 timeout -k 10 600 bash tools/profile.sh || exit 1
cp gpurun_out/prof_r04_s8/pmc_traffic.json $OUT/ && find gpurun_out/prof_r04_s8/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -4 $OUT/kernel_stats.csv; cat $OUT/pmc_traffic.json
