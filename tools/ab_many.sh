#!/bin/bash
# A/B the default build against several exp_*.so on C2 and C4 (run via gpurun)
#   bash tools/ab_many.sh TAG LIB1 [LIB2 ...]
set -o pipefail
TAG=$1; shift
L=$PWD/simple-raytracing-render_amd
ARGS="base:X=0"
for l in "$@"; do ARGS="$ARGS ${l%.so}:SRR_LIB=$L/$l"; done
BENCH_ARGS="" bash tools/ab_libs.sh ${TAG}c2 $ARGS || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh ${TAG}c4 $ARGS || exit 1
