#!/bin/bash
# SQ counters of the chain kernel (where the waves' cycles go): one rocprofv3 --pmc pass per
# counter group, each on a short tools/ab.py run.  Output: gpurun_out/sq/<group>/...
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/sq
mkdir -p "$OUT"
export AB_ROUNDS=${AB_ROUNDS:-3}
VARIANT=${VARIANT:-GE=0}
timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
g=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT"; do
    g=$((g + 1))
    timeout -k 10 200 rocprofv3 --pmc $grp -f csv -d "$OUT/g$g" -o run -- \
        python3 tools/ab.py $VARIANT > "$OUT/g$g.log" 2>&1 || { echo "group $g ($grp) failed"; tail -5 "$OUT/g$g.log"; }
done
python3 tools/sqsum.py "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"
