#!/bin/bash
# Decoded paths after a change of the path kernel: the path tests, then the path pass per kernel.
OUT=${1:-gpurun_out/paths_check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "paths or scope or traceback" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ROUNDS=2 timeout -k 10 300 bash tools/ab_prof.sh $OUT/prof pipe "--steps 10 --warmup 2 --paths" tree
timeout -k 10 300 python3 bench.py --paths --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_paths.json 2> $OUT/bench_paths.err || { tail -5 $OUT/bench_paths.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_paths.json')); r=d['roofline']; print('paths bench', d['ms_per_step'], d['timing']['kernel_ms'], 'frac', r['frac'], 'traffic', r['traffic'], 'golden', d['config']['golden_checked'])"
