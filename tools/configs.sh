#!/bin/bash
# Every BASELINE.json config on one MI355X (run on the GPU box via gpurun), one JSON line each
# under gpurun_out/configs/.  Each GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/configs}
mkdir -p "$OUT"
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
$B --model 100.chmm --ess emit_3_3500_20.ess --steps 50 > "$OUT/c2_100_emit3.json" 2> "$OUT/c2.err" &&
$B --steps 20 > "$OUT/c3_2405_emit50.json" 2> "$OUT/c3.err" &&
$B --steps 10 --paths > "$OUT/c3_2405_emit50_paths.json" 2> "$OUT/c3p.err" &&
$B --steps 20 --level 1 > "$OUT/c4_2405_emit50_spec1.json" 2> "$OUT/c4a.err" &&
$B --steps 3 --warmup 1 --level 2 > "$OUT/c4_2405_emit50_spec2.json" 2> "$OUT/c4b.err" &&
$B --steps 20 --shard covid > "$OUT/c5_2405_covid_1gpu.json" 2> "$OUT/c5.err" &&
$B --steps 5 --warmup 2 --replicate 160 > "$OUT/c3_2405_emit50_x160_wide.json" 2> "$OUT/c3w.err" &&
$B --steps 3 --warmup 1 --replicate 160 --paths --no-pmc > "$OUT/c3_2405_emit50_x160_wide_paths.json" 2> "$OUT/c3wp.err" &&
$B --steps 20 --shard emit50 > "$OUT/c3_2405_emit50_shard_1gpu.json" 2> "$OUT/c3s.err" &&
timeout -k 10 300 python -m spec_viterbi_amd.run_sharded --model data/chmm_files/2405.chmm \
    --ess data/ess_files/covid-19.ess --paths > "$OUT/c5_sharded_1rank_paths.json" 2> "$OUT/c5s.err"
rc=$?
for f in "$OUT"/*.json; do echo "$f: $(cut -c1-400 "$f")"; done
exit $rc
