#!/bin/bash
# Fixed cost of one launch of the diagonal and latency plans: the headline batch truncated to
# 1, 2, 65 and 3500 observations per row, rocprofv3 kernel-trace averages (10 passes each).
set -e
mkdir -p gpurun_out/fixed
for k in diag pipe; do for L in 1 2 65 3500; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/fixed/${k}_$L -o p -- \
        python3 tools/launch.py --kernel $k --maxlen $L --steps 10 > gpurun_out/fixed/${k}_$L.log 2>&1
done; done
