#!/bin/bash
# Round-3 measurements: pipelined parity tests, the headline bench line, the decoded-path bench
# line (pipelined plan), the reference-harness loop over HIP_impl / HIP_spec_impl, and the
# pipelined kernel's wait counters on the headline.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
timeout -k 10 600 python -u -m pytest tests -v -m gpu --maxfail=10 --timeout 120 --timeout-method thread > gpurun_out/r03m/pytest_gpu.log 2>&1; rc=$?; case $rc in 124|134|137|139) exit $rc;; esac
tail -2 gpurun_out/r03m/pytest_gpu.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r03m/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r03m/bench.log | cut -c1-250
timeout -k 10 200 python bench.py --paths --no-pmc --no-cpu-baseline > gpurun_out/r03m/bench_paths.log 2>&1 || exit $?
tail -1 gpurun_out/r03m/bench_paths.log | cut -c1-250
timeout -k 10 300 ./tools/bench_harness --models 100.chmm,1001.chmm,2405.chmm --levels 0,1 > gpurun_out/r03m/harness.jsonl 2> gpurun_out/r03m/harness.err || exit $?
tail -4 gpurun_out/r03m/harness.jsonl
SVH_PIPE_DEBUG=1 timeout -k 10 120 python tools/pipe_dbg.py 2405 emit_50_3500_20 > gpurun_out/r03m/stamps.log 2>&1 || exit $?
head -3 gpurun_out/r03m/stamps.log
