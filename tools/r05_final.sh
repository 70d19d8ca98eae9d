#!/bin/bash
# Round-5 final tree on one MI355X: the whole GPU suite, smoke, the default bench line (PMC passes
# included), every BASELINE config (tools/configs.sh) and a rocprofv3 kernel-trace summary of the
# headline and of the decoded-path pass.  Each GPU step has its own time limit; the first failure ends it.
OUT=${1:-gpurun_out/r05_final}
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_session.sh $OUT || exit 1
OUT=$OUT/configs bash tools/configs.sh > /dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --level 2 > $OUT/configs/c4_2405_emit50_spec2.json 2> $OUT/configs/c4b.err || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_headline -o run -- python3 tools/launch.py --steps 20 --warmup 3 > $OUT/prof_headline.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_paths -o run -- python3 tools/launch.py --steps 10 --warmup 2 --paths > $OUT/prof_paths.log 2>&1 || exit 1
for f in $OUT/configs/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('roofline',{})
print('$(basename $f)', d.get('ms_per_step'), d.get('value'), r.get('frac'), d['config'].get('golden_checked'), d['config'].get('fallback_rows'))" 2>/dev/null || echo "$f: $(head -c 200 $f)"; done
