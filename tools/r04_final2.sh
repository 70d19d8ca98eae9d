#!/bin/bash
# Round 4 final tree, last check: GPU suite, default bench line, bench with decoded paths.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_final}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-700
timeout -k 10 300 python3 bench.py --paths --no-pmc --no-cpu-baseline --steps 10 > $OUT/bench_paths.json 2> $OUT/bench_paths.err || { tail -20 $OUT/bench_paths.err; exit 1; }
tail -1 $OUT/bench_paths.json | cut -c1-700
