#!/bin/bash
# Instruction-cache counters of the headline kernel (one rocprofv3 PMC pass, .txt input).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=${1:-gpurun_out/icache}
mkdir -p $OUT
echo 'pmc: SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES' > $OUT/ic.txt
timeout -s KILL 120 rocprofv3 -i $OUT/ic.txt -f csv -d $OUT/ic -o run -- python3 tools/launch.py --steps 5 --warmup 1 > $OUT/ic.log 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv,glob,sys,collections
f=glob.glob(sys.argv[1]+"/ic/**/*counter_collection.csv",recursive=True)[0]
tot=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open(f)):
    if "pipe_viterbi_kernel" not in r["Kernel_Name"]: continue
    tot[r["Counter_Name"]]+=float(r["Counter_Value"]); n[r["Counter_Name"]]+=1
disp=len(set()) or 1
for k,v in sorted(tot.items()): print(k, v)
PY
