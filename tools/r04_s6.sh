#!/bin/bash
# Round 4 GPU session 6: step table modes 1..4 (TM 3 / 4: packed feeder terms) on the batched
# ring; GPU suite (table-mode test added), A/B, no-exchange step and timeline of modes 3 / 4, the
# one-shot load split.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s6}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=4 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_TM=2 tree:SVH_PIPE_TM=3 tree:SVH_PIPE_TM=4 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for tm in 2 3 4; do
    for d in 1 3; do
        SVH_PIPE_TM=$tm SVH_LIB=build_ab/d/libspec_viterbi_hip.so SVH_PIPE_DEBUG=$d timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tm${tm}_$d.log 2>&1 || { tail $OUT/stamps_tm${tm}_$d.log; exit 1; }
        echo "tm$tm debug=$d: $(grep 'pipe wall' $OUT/stamps_tm${tm}_$d.log | tail -1) | $(grep 'pipe stamps' $OUT/stamps_tm${tm}_$d.log | tail -1)"
    done
done
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py --reps 5 > $OUT/e2e_split.json 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
cat $OUT/e2e_split.json
grep "trace" $OUT/oneshot_trace.log | tail -12
