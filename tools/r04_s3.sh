#!/bin/bash
# Round 4 GPU session 3: GPU suite (wide-plan decoded paths added), step table modes A/B in the
# pipeline, default bench line, wide path batches on the wide plan vs the chain kernel,
# host-to-host split, strong-scaling shares.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 300 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_TM=0 tree:SVH_PIPE_TM=2 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
timeout -k 10 200 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json
for r in 2 8 160; do
  for v in 1 0; do
    SVH_PIPEW_PATHS=$v timeout -k 10 200 python3 tools/launch.py --replicate $r --paths --steps 5 --warmup 1 > $OUT/paths_r${r}_w$v.json 2>&1 || { cat $OUT/paths_r${r}_w$v.json; exit 1; }
    echo "paths x$r wide=$v: $(tail -1 $OUT/paths_r${r}_w$v.json)"
  done
done
timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2>&1 || { cat $OUT/e2e_split.json; exit 1; }
cat $OUT/e2e_split.json
for sh in covid emit50; do
    timeout -k 10 120 python3 tools/shard_shares.py --shard $sh > $OUT/shares_$sh.json 2>&1 || { cat $OUT/shares_$sh.json; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/shares_$sh.json'));print('$sh', {k:(v['makespan_ms'],v['forecast_speedup']) for k,v in d['ranks'].items()})"
done
