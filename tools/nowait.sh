#!/bin/bash
cd "$(dirname "$0")/.."
for cfg in "0 0" "0 16" "4 0" "4 16"; do
  set -- $cfg
  echo -n "GE=$1 dbg=$2: "
  SVH_CHAIN_GE=$1 SVH_BAND_DEBUG=$2 timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-check --kernel 4 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("ms", d["roofline"]["kernel_ms"], "ns/obs", round(d["roofline"]["kernel_ms"]*1e6/3500,1), c["threads"], c["slots"])' || exit 1
done
