# the diagonal plan against the latency and wide pipelined plans by batch width (tools/launch.py):
# where AUTO should switch plans; MODELS="name:ess:widths ..." (widths comma-separated)
set -o pipefail
D=gpurun_out/${OUT:-r06_w}; mkdir -p $D
for spec in ${MODELS:-2405.chmm:emit_50_3500_20.ess:26,50,52,64,90,102}; do
  IFS=: read -r model ess widths <<< "$spec"
  for n in ${widths//,/ }; do for k in diag pipe pipew; do
    timeout -k 10 120 python3 tools/launch.py --model $model --ess $ess --steps 10 --warmup 2 --nseq $n --replicate 200 --kernel $k 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$model', $n, '$k', round(d['kernel_ms_mean'],4), d['golden_ok'])" >> $D/widths.log || echo "$model $n $k rc $?" >> $D/widths.log
  done; done
done
