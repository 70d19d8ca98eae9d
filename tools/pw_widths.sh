#!/bin/bash
# Kernel time of the latency plan, the wide pipelined plan and the chain kernel across batch
# widths (2405.chmm x emit_50_3500_20 replicated with synthetic copies): where AUTO should switch.
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out/${TAG:-pw_widths}.log
: > "$OUT"
for rep in ${REPS:-1 2 3 4 6 8 20 160}; do
    timeout -k 10 200 python tools/pipe_time.py 2405 emit_50_3500_20 5 $rep ${KERNELS:-chain,pipe,pipew} 2>&1 \
        | grep -v amdgpu.ids >> "$OUT" || exit 1
done
