#!/bin/bash
# A/B of an env knob on the C2 bench (run via gpurun): parity first, then
# alternating bench runs with KNOB=0 / KNOB=1.   usage: tools/ab_compact.sh TAG KNOB [bench args]
TAG=${1:-ab}; KNOB=${2:-SRR_COMPACT}; shift 2
O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_paths_match_reference" "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame[default]" \
  > $O/$TAG.tests.log 2>&1 || { tail -30 $O/$TAG.tests.log; exit 1; }
tail -1 $O/$TAG.tests.log
for rep in 1 2; do
  for v in 0 1; do
    env $KNOB=$v timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $O/$TAG.$v.$rep.log 2>&1 || { tail -5 $O/$TAG.$v.$rep.log; exit 1; }
    echo "$KNOB=$v rep $rep: $(grep -o '"value": [0-9.]*' $O/$TAG.$v.$rep.log)"
  done
done
