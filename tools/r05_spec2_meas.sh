#!/bin/bash
# _spec level 2 on chip: the plan/validation tests, the config-4 bench line with its PMC passes on
# the spec2 kernel, a rocprofv3 kernel-trace summary of the same workload, and the reference sweep
# at level 2 (every cell now checked against oracle digests).
OUT=${1:-gpurun_out/spec2m}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    -k "test_errors or spec2_plan" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --level 2 > $OUT/c4_2405_emit50_spec2.json 2> $OUT/c4.err || { tail -5 $OUT/c4.err; exit 1; }
cut -c1-300 $OUT/c4_2405_emit50_spec2.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 tools/launch.py --level 2 --steps 3 --warmup 1 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -4 $OUT/kernel_stats.csv | cut -c1-250
timeout -k 10 600 python3 -u tools/bench_sweep.py --levels 2 --out $OUT/sweep_level2.jsonl > $OUT/sweep.log 2>&1 || { tail -3 $OUT/sweep.log; exit 1; }
python3 -c "
import json, collections
rows = [json.loads(l) for l in open('$OUT/sweep_level2.jsonl')]
print(len(rows), collections.Counter(r['check'] for r in rows))"
