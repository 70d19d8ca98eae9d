# the diagonal plan: the tree against a kept library variant (ab_push/NAME), headline widths; stress
set -o pipefail
D=gpurun_out/${OUT:-r06_d13}; mkdir -p $D
for r in 1 2; do for v in tree ${VARIANTS:-noiw}; do for n in 13 50; do
  if [ $v = tree ]; then lib=spec_viterbi_amd/libspec_viterbi_hip.so; else lib=ab_push/$v/libspec_viterbi_hip.so; fi
  SVH_LIB=$lib timeout -k 10 120 python3 tools/launch.py --steps 10 --warmup 2 --nseq $n 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', $n, round(d['kernel_ms_mean'],4), d['golden_ok'])" >> $D/time.log || echo "$v $n rc $?" >> $D/time.log
done; done; done
timeout -k 10 200 python3 -u tools/diag_stress.py 5 > $D/stress.log 2>&1 || echo "stress rc $?" >> $D/stress.log
