#!/bin/bash
# Config 4 (_spec level 2) on the on-chip kernel: bench line (all 50 rows against the level-2
# digests), the dense-product path for comparison, and a rocprofv3 kernel trace of the level-2 pass.
OUT=${1:-gpurun_out/spec2}
K=${2:-spec2 or level2}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u bench.py --level 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_level2.json 2> $OUT/bench_level2.err || { tail -5 $OUT/bench_level2.err; exit 1; }
cat $OUT/bench_level2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --level 2 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc > $OUT/prof_bench.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -5 $OUT/kernel_stats.csv
