#!/bin/bash
# A/B of an experimental build against the default on C2 and C4 (run via gpurun)
#   bash tools/ab_r3b.sh TAG LIB [LIB2]     (LIB: simple-raytracing-render_amd/exp_*.so)
set -o pipefail
TAG=$1; L=$PWD/simple-raytracing-render_amd
ARGS="base:X=0 exp:SRR_LIB=$L/$2"
[ -n "$3" ] && ARGS="$ARGS exp2:SRR_LIB=$L/$3"
BENCH_ARGS="" bash tools/ab_libs.sh ${TAG}c2 $ARGS || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh ${TAG}c4 $ARGS || exit 1
