#!/bin/bash
# Fixed cost of a diagonal-plan launch, split by ablation builds (ab_push/abN, SVH_DIAG_AB=N):
# the headline batch truncated to one observation per row, rocprofv3 kernel-trace averages.
set -e
D=gpurun_out/fixed_ab_L${L:-1}; mkdir -p $D
for v in ${VARIANTS:-tree ab4 ab5 ab6}; do
    if [ $v = tree ]; then lib=spec_viterbi_amd/libspec_viterbi_hip.so; else lib=ab_push/$v/libspec_viterbi_hip.so; fi
    SVH_LIB=$lib SVH_LAUNCH_NOCHECK=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $D/$v -o p -- \
        python3 tools/launch.py --kernel diag --maxlen ${L:-1} --steps 20 > $D/$v.log 2>&1
done
