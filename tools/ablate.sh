#!/bin/bash
# Timing ablations / stamp breakdowns of the chain kernels (diagnostic).
cd "$(dirname "$0")/.."
for k in ${KERNELS:-4 3}; do
for f in ${FLAGS:-0 4}; do
  echo -n "kernel=$k dbg=$f: "
  SVH_BAND_DEBUG=$f timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-check --kernel $k 2>gpurun_out/ablate_err.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["ms_per_step"], d["roofline"]["kernel_ms"], c["kernel"], c["threads"], c["slots"])' || exit 1
  grep "band stamps" gpurun_out/ablate_err.log | tail -1
done
done
