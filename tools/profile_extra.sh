#!/bin/bash
# rocprofv3 kernel-time summaries of the secondary paths (run on the GPU box via gpurun):
# decoded paths (chain PATHS variant + traceback) and _spec level 2 (dense chunk kernel).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_${TAG}_extra
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/paths" -o run -- \
    python3 bench.py --paths --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/paths.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/spec2" -o run -- \
    python3 bench.py --level 2 --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/spec2.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/spec2_fetch" -o run -- \
    python3 bench.py --level 2 --steps 1 --warmup 0 --no-cpu-baseline --no-check > "$OUT/spec2_fetch.log" 2>&1
