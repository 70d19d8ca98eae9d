#!/bin/bash
# Build a variant of the engine library for A/B timing on the GPU box:
#   tools/ab_build.sh NAME "EXTRA HIPFLAGS"   -> build_ab/NAME/libspec_viterbi_hip.so (AB_ROOT=dir: dir/NAME;
#   build_ab/ stays on this side, .gpurunignore; a library for the GPU box goes to AB_ROOT=ab_push)
# (sources from the tree, e.g. -DSVH_PIPE_HK=0).  Run with SVH_LIB=build_ab/NAME/libspec_viterbi_hip.so.
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2
D=${AB_ROOT:-build_ab}/$NAME
mkdir -p $D/obj
# objects the flags do not change come from the tree's build (make then rebuilds only what differs:
# pass REBUILD=all to build everything with the flags)
if [ -z "$REBUILD" ] && [ -d build ]; then
    # AB_OBJS: the objects the flags change (default: the latency kernel's)
    REB=" ${AB_OBJS:-pipe pipe_tm1 pipe_tm1p} "
    for o in build/*.o; do b=$(basename $o .o); case "$REB" in *" $b "*) ;; *) cp -p $o $D/obj/ ;; esac; done
fi
make -j8 BUILD=$D/obj LIB=$D/libspec_viterbi_hip.so EXTRA_HIPFLAGS="$FLAGS" $D/libspec_viterbi_hip.so > $D/build.log 2>&1
echo "built $D/libspec_viterbi_hip.so"
