timeout -k 10 300 python -u -m pytest tests/test_pipe_gpu.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/pytest_viol.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_viol.log; case $rc in 124|134|137|139) exit $rc;; esac
ROUNDS=3 bash tools/ab_time.sh "--steps 30 --warmup 3" base tree nosleep > gpurun_out/ab3.log 2>&1; cat gpurun_out/ab3.log
bash tools/sq_ab.sh base=build_ab/base/libspec_viterbi_hip.so tree=spec_viterbi_amd/libspec_viterbi_hip.so nosleep=build_ab/nosleep/libspec_viterbi_hip.so > gpurun_out/sq_ab3.log 2>&1; cat gpurun_out/sq_ab3.log
