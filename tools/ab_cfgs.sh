#!/bin/bash
# A/B of library builds / env knobs over several configs (run via gpurun from the repo root):
#   bash tools/ab_cfgs.sh TAG "name:ENV=..;.." ...   (SRR_LIB=... selects a library)
# Configs: C2 (default bench), C1 (30 frames), C4, C5 (one frame each), two alternating passes.
set -o pipefail
TAG=$1; shift
BENCH_ARGS="" bash tools/ab_libs.sh ${TAG}c2 "$@" || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh ${TAG}c1 "$@" || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh ${TAG}c4 "$@" || exit 1
BENCH_ARGS="--scene s5 --steps 1" bash tools/ab_libs.sh ${TAG}c5 "$@" || exit 1
