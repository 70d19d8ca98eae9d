#!/bin/bash
# SQ counters of the pipelined kernel for library variants / diagnostic settings (GPU box):
#   tools/sq_ab.sh NAME=LIB[:ENV=VAL] ...   e.g. base=build_ab/base/libspec_viterbi_hip.so
# One rocprofv3 pass per variant (counters named in a .txt input file: rocprofv3 runs the
# workload as its child), reduced to per-wave, per-observation quad-cycles / instructions.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/sq_ab
mkdir -p $OUT
echo 'pmc: SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY' > $OUT/sq.txt
for spec in "$@"; do
    name=${spec%%=*}; rest=${spec#*=}; lib=${rest%%:*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*:}
    rm -rf $OUT/$name
    env SVH_LIB=$lib $envs timeout -s KILL 120 rocprofv3 -i $OUT/sq.txt -f csv -d $OUT/$name -o run -- \
        python3 tools/launch.py --steps 5 --warmup 1 > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -3 $OUT/$name.log; exit 1; }
    python3 - "$OUT/$name" "$name" <<'PY'
import csv, glob, sys, collections
d, name = sys.argv[1], sys.argv[2]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "pipe_viterbi_kernel" in r["Kernel_Name"]:
            per[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"] or 0)
c = {k: sum(v.values()) / len(v) for k, v in per.items()}
w = c.get("SQ_WAVES", 1) or 1
obs = 3500
print(name, " ".join(f"{k.replace('SQ_','')}={c[k]/w/obs:.2f}" for k in sorted(c) if k != "SQ_WAVES"), f"waves={w:.0f}")
PY
done
