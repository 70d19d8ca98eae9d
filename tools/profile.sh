#!/bin/bash
# rocprofv3 evidence for the bench's dominant kernel (run on the GPU box via gpurun):
#   1. --kernel-trace --stats (CSV): per-kernel average duration,
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE in separate passes (they do not fit one pass),
# then tools/pmc_traffic.py turns them into HBM bytes per launch (gfx950 corrections applied).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_${TAG}
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 2 --no-cpu-baseline"}
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/trace" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/fetch" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/write" -o run -- \
    python3 bench.py $ARGS > "$OUT/bench_write.log" 2>&1 &&
python3 tools/pmc_traffic.py "$OUT" > "$OUT/pmc_traffic.json"
