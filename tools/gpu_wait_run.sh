#!/bin/bash
# Run one gpurun command, retrying only while the call is refused for infrastructure reasons
# before anything ran (status "transient": no free box, box lost while being prepared, backoff);
# waits as long as gpurun's "retry in N s" asks.  A call that ran -- whatever its outcome -- is
# never repeated.  Log: gpurun_out/wait_run.log
#   tools/gpu_wait_run.sh TIMEOUT 'COMMAND'
cd "$(dirname "$0")/.."
T=$1; CMD=$2
for i in $(seq 1 40); do
    /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > gpurun_out/wait_run.log 2>&1
    st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
    if [ "$st" != "transient" ]; then echo "attempt $i: status $st" >> gpurun_out/wait_run.log; exit 0; fi
    w=$(grep -o "retry in [0-9]*s" gpurun_out/wait_run.log | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-170} + 15 ))
done
