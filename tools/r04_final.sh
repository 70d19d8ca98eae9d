#!/bin/bash
# Round 4 final tree on MI355X: smoke, every BASELINE config (tools/configs.sh), host-to-host split,
# strong-scaling shares.  Outputs under gpurun_out/r04_final (copied to profiles/r04_final).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_final}
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
OUT=$OUT timeout -k 10 900 bash tools/configs.sh > $OUT/configs.log 2>&1 || { tail -30 $OUT/configs.log; exit 1; }
cut -c1-300 $OUT/configs.log
SVH_TRACE_ONESHOT=1 timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2> $OUT/oneshot_trace.log || { tail $OUT/oneshot_trace.log; exit 1; }
cat $OUT/e2e_split.json
for sh in covid emit50; do
    timeout -k 10 120 python3 tools/shard_shares.py --shard $sh > $OUT/shares_$sh.json 2> $OUT/shares_$sh.err || { cat $OUT/shares_$sh.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/shares_$sh.json'));print('$sh', {k:(v['makespan_ms'],v['forecast_speedup']) for k,v in d['ranks'].items()})"
done
