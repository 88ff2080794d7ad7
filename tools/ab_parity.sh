#!/bin/bash
# parity subset on the default build, then A/B default vs LIB on C1, C2, C4 (run via gpurun)
#   bash tools/ab_parity.sh TAG LIB [LIB2]
set -o pipefail
TAG=$1; L=$PWD/simple-raytracing-render_amd; O=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_paths_match_reference" "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame" \
  > $O/$TAG.tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 $O/$TAG.tests.log; [ $rc -eq 0 ] || exit 1
fi
ARGS="new:X=0 old:SRR_LIB=$L/$2"
[ -n "$3" ] && ARGS="$ARGS old2:SRR_LIB=$L/$3"
BENCH_ARGS="--scene s1 --steps 20 --warmup 3" bash tools/ab_libs.sh ${TAG}c1 $ARGS || exit 1
BENCH_ARGS="" bash tools/ab_libs.sh ${TAG}c2 $ARGS || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh ${TAG}c4 $ARGS || exit 1
