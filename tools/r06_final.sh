#!/bin/bash
# Round-6 closing pass on one MI355X: the whole-tree measurement (tools/measure_all.sh), then the
# diagonal plan's finish-kernel variant (ab_push/finish, SVH_DIAG_FINISH=1) through its parity tests
# and the fixed-cost A/B (tools/diag_fixed_ab.sh).  The first failure ends it.
set -o pipefail
bash tools/measure_all.sh gpurun_out/r06_final || exit 1
SVH_LIB=ab_push/finish/libspec_viterbi_hip.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_diag_gpu.py tests/test_spec_gpu.py tests/test_gpu_parity.py > gpurun_out/r06_final/finish_pytest.log 2>&1 || exit 1
VARIANTS="tree finish atompad ab7 ab8" L=1 bash tools/diag_fixed_ab.sh || exit 1
VARIANTS="tree finish atompad" L=3500 bash tools/diag_fixed_ab.sh
