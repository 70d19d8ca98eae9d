#!/bin/bash
# rocprofv3 evidence for the chain kernel's roofline (run on the GPU box via gpurun):
# per workload, one --kernel-trace --stats pass, two SQ counter passes (VALU issue, wait split)
# and separate FETCH_SIZE / WRITE_SIZE passes; tools/sq_summary.py reduces them to JSON.
#   TAG=r02 WORKLOADS="narrow wide" tools/sq_profile.sh   (SQ3=1: an LDS counter pass as well)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/sq_${TAG}
mkdir -p "$OUT"
run() {  # name, pass, rocprof args..., -- launch args
    local name=$1 pass=$2; shift 2
    local prof=() ; while [ "$1" != "--" ]; do prof+=("$1"); shift; done; shift
    timeout -s KILL 120 rocprofv3 "${prof[@]}" -f csv -d "$OUT/$name/$pass" -o run -- \
        python3 tools/launch.py "$@" > "$OUT/$name/$pass.log" 2>&1
}
for w in ${WORKLOADS:-narrow wide}; do
    case $w in
        narrow) ARGS="--steps 5 --warmup 1" ;;
        wide)   ARGS="--replicate 160 --steps 3 --warmup 1" ;;
        covid)  ARGS="--ess covid-19.ess --steps 5 --warmup 1" ;;
        *) ARGS="$w" ;;
    esac
    mkdir -p "$OUT/$w"
    run $w trace --kernel-trace --stats -- $ARGS &&
    run $w sq1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -- $ARGS &&
    run $w sq2 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -- $ARGS &&
    { [ -z "$SQ3" ] || run $w sq3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL -- $ARGS; } &&
    run $w fetch --pmc FETCH_SIZE -- $ARGS &&
    run $w write --pmc WRITE_SIZE -- $ARGS || { echo "workload $w failed"; exit 1; }
    python3 tools/sq_summary.py "$OUT/$w" > "$OUT/$w/summary.json" && cat "$OUT/$w/summary.json"
done
