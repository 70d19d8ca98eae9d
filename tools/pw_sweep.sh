#!/bin/bash
# A/B timings of the wide pipelined plan on 2405 x emit_50 x160 (8000 sequences); each line runs
# tools/pipe_time.py with one setting.  SVH_PIPE_DEBUG=N sets diagnostic bits N>>1 (wide kernel:
# 1 = no boundary exchange, 2 = packed f32 adds).
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pw}.log
: > "$OUT"
for setting in "${@:-}"; do
    env $setting timeout -k 10 200 python tools/pipe_time.py 2405 emit_50_3500_20 3 160 ${KERNELS:-pipew} \
        2>&1 | grep -v amdgpu.ids | sed "s|^|[$setting] |" >> "$OUT" || exit 1
done
