#!/bin/bash
# The headline's wait split: per role (workgroup g, wave w) the diagnostic
# build's wait counters and re-read groups averaged over all 50 rows; the bench line with its SQ,
# HBM and LDS PMC passes; the per-kernel time of the tree, of every exchange operation without a
# wait (nowait) and of no exchange at all (diagnostic sweep without boundary roles).
OUT=${1:-gpurun_out/waitsplit}
mkdir -p $OUT
export TMPDIR=/tmp
SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --steps 2 --warmup 1 > $OUT/stamps.log 2>&1 || { tail -5 $OUT/stamps.log; exit 1; }
grep -A 25 "wait split by role" $OUT/stamps.log | head -24
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], json.dumps(d['roofline'].get('lds')), d['roofline'].get('cycle_split'))"
ROUNDS=2 timeout -k 10 400 bash tools/ab_prof.sh $OUT/split pipe_viterbi "--steps 10 --warmup 2" tree nowait diag:SVH_PIPE_DEBUG=3 > $OUT/split.log 2>&1 || { cat $OUT/split.log; exit 1; }
cat $OUT/split.log
