#!/bin/bash
# Round 4 GPU session: GPU test suite on the tree, A/B of the step table modes and knobs, the
# no-exchange step of diagnostic builds, the host-to-host split.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/r04_s1}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
ROUNDS=3 timeout -k 10 400 bash tools/ab_time.sh "--steps 30 --warmup 3" tree tree:SVH_PIPE_TM=0 tree:SVH_PIPE_TM=2 t4r t4rp > $OUT/ab.log 2>&1 || { cat $OUT/ab.log; exit 1; }
cat $OUT/ab.log
for v in t0d t4d; do
    SVH_LIB=build_ab/$v/libspec_viterbi_hip.so SVH_PIPE_DEBUG=3 timeout -k 10 120 python3 tools/launch.py --steps 1 --warmup 1 > $OUT/stamps_${v}_3.log 2>&1 || exit $?
    echo "$v no-exchange: $(grep 'pipe wall' $OUT/stamps_${v}_3.log | tail -1)"
done
timeout -k 10 60 tools/ubench/step_ubench 250 > $OUT/step_ubench.txt 2>&1 && cat $OUT/step_ubench.txt
timeout -k 10 120 python3 tools/e2e_split.py > $OUT/e2e_split.json 2>&1 || { cat $OUT/e2e_split.json; exit 1; }
cat $OUT/e2e_split.json
for sh in covid emit50; do
    timeout -k 10 120 python3 tools/shard_shares.py --shard $sh > $OUT/shares_$sh.json 2>&1 || { cat $OUT/shares_$sh.json; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/shares_$sh.json'));print('$sh', {k:(v['makespan_ms'],v['forecast_speedup']) for k,v in d['ranks'].items()})"
done
