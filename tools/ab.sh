#!/bin/bash
# One parametrised A/B run on a GPU box (via gpurun, from the repo root):
#
#   bash tools/ab.sh TAG [-t TESTLIB]... [-c "c2 c1 c3 c4 c4r c5 d100"] [-p] name:ENV;ENV ...
#
#   -t LIB   first run the GPU tests against that library (SRR_LIB=LIB; "head" = the in-tree
#            libsrr.so): a variant is only timed once it is bit-exact
#   -c CFGS  configs to time (default "c2 c1 c4 c5"): each as an alternating two-pass
#            tools/ab_libs.sh over every variant
#   -p       also record the phase timing of C2 / C4 / C4_real with the diagnostics build
#   variants: a label, then space-free env assignments separated by ';'
#            (SRR_LIB=simple-raytracing-render_amd/exp_x.so selects a library; X=0 is a no-op)
# Output: gpurun_out/TAG*.log, one "name rep N: value" line per run on stdout.
set -o pipefail
TAG=$1; shift
TESTS=(); CFGS="c2 c1 c4 c5"; PHASES=0
while getopts "t:c:p" o; do
  case $o in t) TESTS+=("$OPTARG");; c) CFGS=$OPTARG;; p) PHASES=1;; *) exit 2;; esac
done
shift $((OPTIND - 1))
L=$PWD/simple-raytracing-render_amd
for lib in "${TESTS[@]}"; do
  env_lib=""; [ "$lib" != head ] && env_lib="SRR_LIB=$lib"
  env $env_lib timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    > gpurun_out/$TAG.tests.$(basename $lib).log 2>&1
  rc=$?; tail -1 gpurun_out/$TAG.tests.$(basename $lib).log; [ $rc -eq 0 ] || exit 1
done
declare -A ARGS=([c2]="" [c1]="--scene s1 --steps 30 --warmup 3" [c3]="--scene s3 --steps 2"
                 [c3m]="--scene s3_metal --steps 2" [c4]="--scene s4 --steps 2" [c5]="--scene s5 --steps 1"
                 [c4r]="--scene s4_real --steps 1" [d100]="--scene s2 --divs 100")
for c in $CFGS; do
  BENCH_ARGS="${ARGS[$c]}" bash tools/ab_libs.sh $TAG$c "$@" || exit 1
done
if [ $PHASES = 1 ]; then
  for a in "" "--scene s4 --steps 1" "--scene s4_real --steps 1"; do
    t=$(echo "x$a" | tr -c 'a-z0-9' '_')
    SRR_LIB=$L/libsrr_diag.so SRR_PATHS_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline \
      --warmup 1 --steps 1 $a > gpurun_out/$TAG.timing$t.log 2>&1 || exit 1
    echo "$a"; grep -h "per wave-iteration\|mixture loop" gpurun_out/$TAG.timing$t.log | tail -2
  done
fi
