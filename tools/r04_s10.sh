#!/bin/bash
# Round 4 GPU session 10: XCD-local hand-offs the default (SVH_PIPE_XL), rows mapped to
# workgroups by XCD class (SVH_PIPE_XMAP, run-time A/B).  GPU suite, A/B, placement-tagged
# timelines, bench line, rocprofv3 stats + PMC.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s10}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
SVH_PIPE_XMAP=0 timeout -k 10 300 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread -k "headline or table_modes or lengths or covid" > $OUT/pytest_xmap0.log 2>&1; rc=$?
tail -2 $OUT/pytest_xmap0.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=4 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_XMAP=0 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for xm in 1 0; do
    SVH_PIPE_XMAP=$xm SVH_LIB=build_ab/d/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_xmap$xm.log 2>&1 || { tail $OUT/stamps_xmap$xm.log; exit 1; }
    echo "xmap $xm: $(grep 'pipe wall' $OUT/stamps_xmap$xm.log | tail -1)"
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-900
TAG=r04_s10 timeout -k 10 600 bash tools/profile.sh || exit 1
cp gpurun_out/prof_r04_s10/pmc_traffic.json $OUT/ && find gpurun_out/prof_r04_s10/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -4 $OUT/kernel_stats.csv
