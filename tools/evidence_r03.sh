#!/bin/bash
# Round-3 evidence on one GPU box (run via gpurun from the repo root):
#   GPU tests -> counters (tools/counters.sh) -> FETCH/WRITE passes -> bench line with
#   cpu_baseline -> rocprofv3 kernel-trace --stats of the same bench command.
# usage: tools/evidence_r03.sh TAG [SCENE]   (outputs gpurun_out/TAG.*)
set -o pipefail
TAG=${1:-ev}
SCENE=${2:-s2}
R=$PWD
O=$R/gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/$TAG.tests.log 2>&1 || { tail -20 $O/$TAG.tests.log; exit 1; }
  tail -1 $O/$TAG.tests.log
fi
bash tools/counters.sh ${TAG}_cnt --scene $SCENE > $O/$TAG.counters.log 2>&1 || { tail -5 $O/$TAG.counters.log; exit 1; }
echo "counters ok"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/$TAG.pmc_$c -o run -- \
    python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --scene $SCENE > $O/$TAG.pmc_$c.log 2>&1 \
    || { echo "pmc $c failed"; tail -5 $O/$TAG.pmc_$c.log; exit 1; }
done
python $R/tools/pmc_traffic.py $O/$TAG.pmc_FETCH_SIZE $O/$TAG.pmc_WRITE_SIZE k_paths $O/$TAG.pmc_$SCENE.json || exit 1
cd $R
timeout -k 10 600 python bench.py --scene $SCENE > $O/$TAG.bench.log 2>&1 || { tail -5 $O/$TAG.bench.log; exit 1; }
grep '^{' $O/$TAG.bench.log | cut -c1-300
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$TAG.prof -o run --output-format csv -- \
  python $R/bench.py --no-cpu-baseline --scene $SCENE > $O/$TAG.prof.log 2>&1 || { tail -5 $O/$TAG.prof.log; exit 1; }
grep '^{' $O/$TAG.prof.log | cut -c1-200
python $R/tools/stats.py $O/$TAG.prof
