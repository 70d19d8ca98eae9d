#!/bin/bash
# Chain kernel: emission table in VGPRs vs streamed from L2 at several wave counts (diagnostic).
cd "$(dirname "$0")/.."
for ge in ${GES:-0 4 8 2}; do
  echo -n "SVH_CHAIN_GE=$ge: "
  SVH_CHAIN_GE=$ge timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${CHECK:-} --kernel 4 2>gpurun_out/ge_err.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("ms", d["roofline"]["kernel_ms"], "ns/obs", round(d["roofline"]["kernel_ms"]*1e6/3500,1), c["kernel"], c["threads"], c["slots"])' || { tail -3 gpurun_out/ge_err.log; exit 1; }
done
