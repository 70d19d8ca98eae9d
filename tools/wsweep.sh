#!/bin/bash
# Per-observation time of the chain kernel vs workgroup width (diagnostic).
cd "$(dirname "$0")/.."
for mdl in ${MODELS:-300.chmm 600.chmm 1200.chmm 2405.chmm}; do
for f in ${FLAGS:-0}; do
  echo -n "$mdl dbg=$f: "
  SVH_BAND_DEBUG=$f timeout -k 10 120 python bench.py --model $mdl --steps 10 --warmup 2 --no-cpu-baseline --no-check --kernel ${KERNEL:-4} 2>gpurun_out/wsweep_err.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print("ms", d["roofline"]["kernel_ms"], "ns/obs", round(d["roofline"]["kernel_ms"]*1e6/3500,1), c["kernel"], c["threads"], c["slots"])' || exit 1
  grep "band stamps" gpurun_out/wsweep_err.log | tail -1
done
done
