#!/bin/bash
# Round-3 (session 2) probe on one GPU box, from the repo root:
#   GPU tests -> C2 bench -> per-phase timing of C1/C2/C4/C5 -> CBVH/QUAD A/B on C4.
# usage: bash tools/probe_r3b.sh TAG     (outputs gpurun_out/TAG.*)
set -o pipefail
TAG=${1:-pb}
O=gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/$TAG.tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 $O/$TAG.tests.log; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/$TAG.bench.log 2>&1 || { tail -5 $O/$TAG.bench.log; exit 1; }
grep '^{' $O/$TAG.bench.log | cut -c1-300
for s in s1 s2 s4 s5; do
  SRR_PATHS_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 1 --warmup 0 --scene $s > $O/$TAG.tim_$s.log 2>&1 || { tail -5 $O/$TAG.tim_$s.log; exit 1; }
  echo "$s: $(grep -A1 'per wave-iteration' $O/$TAG.tim_$s.log | tr '\n' ' ')"
done
for env in "SRR_CBVH=0" "SRR_CBVH=1" "SRR_QUAD=1"; do
  env $env timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --scene s4 > $O/$TAG.ab_s4_$env.log 2>&1 || { tail -5 $O/$TAG.ab_s4_$env.log; exit 1; }
  echo "s4 $env: $(grep '^{' $O/$TAG.ab_s4_$env.log | cut -c1-120)"
done
