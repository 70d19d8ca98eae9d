set -e
export TMPDIR=/tmp
OUT=gpurun_out/r05_s5; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "spec" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
SVH_LIB=build_ab/s2diag/libspec_viterbi_hip.so SVH_SPEC2_DEBUG=1 timeout -k 10 120 python3 tools/launch.py --level 2 --steps 1 --warmup 0 > $OUT/diag.log 2>&1
cat $OUT/diag.log
timeout -k 10 120 python3 tools/launch.py --level 2 --steps 10 --warmup 2 > $OUT/launch.log 2>&1
cat $OUT/launch.log
