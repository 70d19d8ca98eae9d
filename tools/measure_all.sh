#!/bin/bash
# Whole-tree measurement on one MI355X (run on the GPU box via gpurun): the GPU suite, smoke, the
# default bench line (PMC passes included), every BASELINE config (tools/configs.sh), the latency
# plan at two workgroups per CU (the headline file twice, golden-checked rows), and rocprofv3
# kernel-trace summaries of the headline, the decoded-path pass and the level-2 pass.  Each GPU step
# has its own time limit; the first failure ends it.  Usage: bash tools/measure_all.sh <outdir>
OUT=${1:-gpurun_out/measure}
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu_session.sh $OUT || exit 1
OUT=$OUT/configs bash tools/configs.sh > /dev/null || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 20 --replicate 2 > $OUT/configs/c3_2405_emit50_x2_latency.json 2> $OUT/configs/c3x2.err || exit 1
for w in headline:"" paths:"--paths" level2:"--level 2"; do
  name=${w%%:*}; args=${w#*:}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_$name -o run -- python3 bench.py --steps 20 --warmup 3 --no-pmc --no-cpu-baseline $args > $OUT/prof_$name.json 2> $OUT/prof_$name.err || exit 1
done
for f in $OUT/configs/*.json; do python3 -c "
import json,sys
d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d.get('roofline',{})
print('$(basename $f)', d.get('ms_per_step'), d.get('value'), r.get('frac'), d['config'].get('golden_checked'), d['config'].get('fallback_rows'))" 2>/dev/null || echo "$f: $(head -c 200 $f)"; done
