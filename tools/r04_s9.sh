#!/bin/bash
# Round 4 GPU session 9: exchange LDS reads kept in place (SVH_PIPE_LDSX, tree default) vs not
# (ldsx0), XCD-local granule / progress stores (xl1), with placement-tagged timelines of both.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s9}
mkdir -p $OUT
if [ -z "$SKIP_SUITE" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
fi
# the XCD-local variant on the parity tests of the latency plan first (a wrong hand-off would show
# as a bounded-wait give-up or a digest mismatch)
SVH_LIB=build_ab/xl1/libspec_viterbi_hip.so timeout -k 10 300 python -u -m pytest tests/test_pipe_gpu.py -x -q --timeout 120 --timeout-method thread -k "(headline or table_modes or long_sequence or covid_ragged or test_pipe_sequence_lengths) and not paths" > $OUT/pytest_xl1.log 2>&1; rc=$?
tail -3 $OUT/pytest_xl1.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=4 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree ldsx0 xl1 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in d xl1d; do
    SVH_LIB=build_ab/$v/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_$v.log 2>&1 || { tail $OUT/stamps_$v.log; exit 1; }
    echo "$v: $(grep 'pipe wall' $OUT/stamps_$v.log | tail -1)"
done
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-900
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
cat $OUT/e2e_split.json
