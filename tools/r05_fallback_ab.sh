#!/bin/bash
# (1) the headline pass with and without its second launch (the serial fallback that exits at once
#     unless a row failed its speculation check; SVH_PIPE_SKIP_FALLBACK=1 is diagnostics only), by
#     events and by the bench's wall clock; stamps of both (per-XCD entry times).
# (2) latency plan vs wide plan for 100 / 150 / 200 sequences (AUTO's threshold).
OUT=${1:-gpurun_out/fallback_ab}
mkdir -p $OUT
export TMPDIR=/tmp
ROUNDS=3 timeout -k 10 300 bash tools/ab_time.sh "--steps 20 --warmup 3" tree tree:SVH_PIPE_SKIP_FALLBACK=1 > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in 0 1; do
  SVH_PIPE_SKIP_FALLBACK=$v timeout -k 10 300 python3 bench.py --steps 50 --warmup 5 --no-pmc --no-cpu-baseline > $OUT/bench_skip$v.json 2> $OUT/bench_skip$v.err || { tail -3 $OUT/bench_skip$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_skip$v.json')); print('bench skip=$v', d['ms_per_step'], d['timing']['kernel_ms'])"
  SVH_LIB=build_ab/diag/libspec_viterbi_hip.so SVH_PIPE_DEBUG=1 SVH_PIPE_SKIP_FALLBACK=$v timeout -k 10 120 python3 tools/launch.py --steps 3 --warmup 3 > $OUT/stamps_skip$v.log 2>&1
  grep -h "last sweep" $OUT/stamps_skip$v.log | tail -1
  grep -h " seq " $OUT/stamps_skip$v.log | tail -50 | python3 -c "
import sys,re,collections
d=collections.defaultdict(list)
for l in sys.stdin:
    for m in re.finditer(r'in ([0-9.]+) st [0-9.]+ end ([0-9.]+) x(\d)', l): d[int(m.group(3))].append((float(m.group(1)), float(m.group(2))))
print('skip=$v entry/end by XCD:', {x: (round(min(a for a,b in v),1), round(max(b for a,b in v),1)) for x,v in sorted(d.items())})"
done
for n in 100 150 200; do
  r=$((n/50))
  SVH_PIPE_MAX_NSEQ=$n SVH_LAUNCH_NOCHECK=1 timeout -k 10 120 python3 tools/launch.py --replicate $r --steps 10 --warmup 2 > $OUT/lat$n.json 2>&1
  timeout -k 10 120 python3 tools/launch.py --replicate $r --steps 10 --warmup 2 > $OUT/auto$n.json 2>&1
  python3 -c "import json; a=json.loads(open('$OUT/lat$n.json').read().strip().splitlines()[-1]); b=json.loads(open('$OUT/auto$n.json').read().strip().splitlines()[-1]); print('nseq $n latency', round(a['kernel_ms_mean'],4), 'auto(wide)', round(b['kernel_ms_mean'],4))"
done
