#!/bin/bash
# Round 4 GPU session 5: the tree with the batched LDS ring on the pair-table kernels.  GPU suite,
# A/B of the table modes, the diagnostic build's no-exchange step and timeline, the bench line,
# rocprofv3 kernel stats + PMC traffic, the one-shot host-to-host trace, latency-plan geometries
# for few-sequence batches, strong-scaling shares.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s5}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 300 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_TM=0 tree:SVH_PIPE_TM=2 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for tm in 1 2; do
    for d in 1 3; do
        SVH_PIPE_TM=$tm SVH_LIB=build_ab/d/libspec_viterbi_hip.so SVH_PIPE_DEBUG=$d timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_tm${tm}_$d.log 2>&1 || { tail $OUT/stamps_tm${tm}_$d.log; exit 1; }
        echo "tm$tm debug=$d: $(grep 'pipe wall' $OUT/stamps_tm${tm}_$d.log | tail -1) | $(grep 'pipe stamps' $OUT/stamps_tm${tm}_$d.log | tail -1)"
    done
done
timeout -k 10 200 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
TAG=r04_s5 timeout -k 10 900 bash tools/profile.sh || exit 1
cp -r gpurun_out/prof_r04_s5/pmc_traffic.json $OUT/ && find gpurun_out/prof_r04_s5/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -5 $OUT/kernel_stats.csv; cat $OUT/pmc_traffic.json
timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2> $OUT/e2e_split.err || { cat $OUT/e2e_split.err; exit 1; }
cat $OUT/e2e_split.json
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py --reps 5 > /dev/null 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
grep "oneshot trace" $OUT/oneshot_trace.log | tail -8
timeout -k 10 300 python3 tools/geom_sweep.py > $OUT/geom_covid.jsonl 2> $OUT/geom_covid.err || { tail $OUT/geom_covid.err; exit 1; }
head -5 $OUT/geom_covid.jsonl
for sh in covid emit50; do
    timeout -k 10 120 python3 tools/shard_shares.py --shard $sh > $OUT/shares_$sh.json 2> $OUT/shares_$sh.err || { cat $OUT/shares_$sh.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/shares_$sh.json'));print('$sh', {k:(v['makespan_ms'],v['forecast_speedup']) for k,v in d['ranks'].items()})"
done
