#!/bin/bash
# Decoded paths on the latency plan: the pass with and without the per-step LDS record store
# (-DSVH_PIPE_NO_PRING: ablation, wrong paths), per kernel under rocprofv3.
OUT=${1:-gpurun_out/paths_ab}
mkdir -p $OUT
ROUNDS=2 timeout -k 10 500 bash tools/ab_prof.sh $OUT pipe_viterbi_kernel "--steps 10 --warmup 2 --paths" tree nopring
