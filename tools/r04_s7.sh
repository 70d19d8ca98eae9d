#!/bin/bash
# Round 4 GPU session 7: TM = 4 the default (scores and decoded paths), vectorised symbol packing.
# GPU suite, A/B of the granule knobs (prefetch depth 4, store step 0 / 4) against the tree,
# placement-tagged timeline, bench line, one-shot trace, path variants TM 4 vs 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s7}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree gpf4 gst0 gst4 tree:SVH_PIPE_TM=2 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for d in 1 3; do
    SVH_LIB=build_ab/d/libspec_viterbi_hip.so SVH_PIPE_DEBUG=$d timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tm4_$d.log 2>&1 || { tail $OUT/stamps_tm4_$d.log; exit 1; }
    echo "tm4 debug=$d: $(grep 'pipe wall' $OUT/stamps_tm4_$d.log | tail -1)"
done
for tm in 4 1; do
    SVH_PIPE_TM=$tm timeout -k 10 120 python3 tools/launch.py --paths --steps 10 --warmup 2 > $OUT/paths_tm$tm.json 2>&1 || { tail $OUT/paths_tm$tm.json; exit 1; }
    echo "paths tm$tm: $(tail -1 $OUT/paths_tm$tm.json | cut -c1-200)"
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-1200
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py --reps 5 > $OUT/e2e_split.json 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
cat $OUT/e2e_split.json
grep "trace" $OUT/oneshot_trace.log | tail -6
