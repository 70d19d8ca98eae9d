#!/bin/bash
# Interleaved A/B timing of library variants (tools/ab_build.sh) on the GPU box: for each round,
# each variant runs tools/launch.py in its own process; prints the mean HIP-event time per pass
# (golden-checked on the headline workload).
#   tools/ab_time.sh "ARGS for launch.py" VARIANT...
# VARIANT = LIB[:ENV=VALUE[,ENV=VALUE...]]: LIB a name under build_ab or "tree" (the in-tree
# library), then environment settings for that run (e.g. tree:SVH_PIPE_TM=0).
set -o pipefail
cd "$(dirname "$0")/.."
ARGS=$1; shift
ROUNDS=${ROUNDS:-3}
for r in $(seq $ROUNDS); do
    for v in "$@"; do
        name=${v%%:*}; envs=""
        [ "$name" != "$v" ] && envs=${v#*:}
        if [ "$name" = tree ]; then lib=spec_viterbi_amd/libspec_viterbi_hip.so; else lib=build_ab/$name/libspec_viterbi_hip.so; fi
        out=$(env SVH_LIB=$lib ${envs//,/ } timeout -k 10 120 python3 tools/launch.py $ARGS 2>/dev/null) || { echo "$v failed ($?)"; exit 1; }
        echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', 'round $r', round(d['kernel_ms_mean'],4), 'golden', d['golden_ok'])"
    done
done
