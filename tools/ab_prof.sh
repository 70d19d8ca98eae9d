#!/bin/bash
# Per-kernel A/B timing of library variants under rocprofv3 (kernel trace): the average duration of
# the kernels whose name contains PATTERN, per variant and round (interleaved), so a variant whose
# results fall back to another kernel (ablations) is still timed on the kernel itself.
#   tools/ab_prof.sh OUTDIR PATTERN "ARGS for launch.py" VARIANT...   (VARIANT as in tools/ab_time.sh)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=$1; PAT=$2; ARGS=$3; shift 3
ROUNDS=${ROUNDS:-2}
export TMPDIR=/tmp
mkdir -p $OUT
for r in $(seq $ROUNDS); do
    for v in "$@"; do
        name=${v%%:*}; envs=""
        [ "$name" != "$v" ] && envs=${v#*:}
        if [ "$name" = tree ]; then lib=spec_viterbi_amd/libspec_viterbi_hip.so; else lib=build_ab/$name/libspec_viterbi_hip.so; fi
        d=$OUT/${v//[:=,]/_}_r$r
        env SVH_LIB=$lib SVH_LAUNCH_NOCHECK=1 ${envs//,/ } timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $d -o run -- python3 tools/launch.py $ARGS > $d.log 2>&1 || { echo "$v failed"; tail -5 $d.log; exit 1; }
        f=$(find $d -name "*kernel_stats.csv" | head -1)
        python3 - "$f" "$PAT" "$v" "$r" <<'PY'
import csv, sys
f, pat, v, r = sys.argv[1:]
for row in csv.DictReader(open(f)):
    if pat in row["Name"]:
        print(f"{v} round {r}: {float(row['AverageNs'])/1e3:.2f} us x{row['Calls']}  {row['Name'][:90]}")
PY
    done
done
