#!/bin/bash
# Two latency-plan workgroups per CU: the headline file twice (100 sequences, 500 workgroups of 4
# waves on 256 CUs) on the latency plan (SVH_PIPE_MAX_NSEQ=100) against the headline (50).  Per-row
# start / end times from the diagnostic build show whether rows whose CUs hold two workgroups run
# slower.
OUT=${1:-gpurun_out/occ2}
mkdir -p $OUT
export TMPDIR=/tmp
L=build_ab/gx2/libspec_viterbi_hip.so
D=build_ab/diaggx2/libspec_viterbi_hip.so
for r in 1 2; do
  SVH_LIB=$L timeout -k 10 120 python3 tools/launch.py --steps 20 --warmup 3 > $OUT/l50_$r.json 2>&1
  SVH_LIB=$L SVH_PIPE_MAX_NSEQ=100 SVH_LAUNCH_NOCHECK=1 timeout -k 10 120 python3 tools/launch.py --replicate 2 --steps 20 --warmup 3 > $OUT/l100_$r.json 2>&1
  SVH_LIB=$L timeout -k 10 120 python3 tools/launch.py --replicate 2 --steps 20 --warmup 3 > $OUT/w100_$r.json 2>&1
  for f in l50 l100 w100; do python3 -c "import json,sys; d=json.loads(open('$OUT/${f}_$r.json').read().strip().splitlines()[-1]); print('$f', round(d['kernel_ms_mean'],4), d['info']['pipe_groups'], d['golden_ok'])"; done
done
SVH_LIB=$D SVH_PIPE_DEBUG=1 SVH_PIPE_MAX_NSEQ=100 timeout -k 10 120 python3 tools/launch.py --replicate 2 --steps 1 --warmup 1 > $OUT/stamps100.log 2>&1
grep -h "pipe stamps\|last sweep" $OUT/stamps100.log
