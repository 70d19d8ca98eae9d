#!/bin/bash
# Build variant libraries of the engine from alternative chain_impl.h files for A/B timing:
#   tools/ab_lib.sh NAME path/to/chain_impl.h   -> build_ab/NAME/libspec_viterbi_hip.so
# (other sources from the tree).  Run with SVH_LIB=build_ab/NAME/libspec_viterbi_hip.so.
set -e
cd "$(dirname "$0")/.."
NAME=$1; HDR=$2
D=build_ab/$NAME
mkdir -p $D/src
cp spec_viterbi_amd/csrc/* $D/src/
cp "$HDR" $D/src/chain_impl.h
make -j16 CSRC=$D/src BUILD=$D/obj LIB=$D/libspec_viterbi_hip.so $D/libspec_viterbi_hip.so > $D/build.log 2>&1
echo "built $D/libspec_viterbi_hip.so"
