#!/bin/bash
# Round evidence on one GPU box (run via gpurun from the repo root):
#   GPU parity tests -> PMC FETCH/WRITE passes on the trace kernel -> full default
#   bench line (with cpu_baseline) -> kernel-trace --stats profile of the same command.
# usage: tools/evidence.sh TAG [SCENE]
set -o pipefail
TAG=${1:-r01}
SCENE=${2:-s2}
R=$PWD
O=$R/gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/$TAG.tests.log 2>&1 || { tail -20 $O/$TAG.tests.log; exit 1; }
tail -1 $O/$TAG.tests.log
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/$TAG.pmc_$c -o run -- \
    python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --scene $SCENE > $O/$TAG.pmc_$c.log 2>&1 \
    || { echo "pmc $c failed"; tail -5 $O/$TAG.pmc_$c.log; exit 1; }
done
python $R/tools/pmc_traffic.py $O/$TAG.pmc_FETCH_SIZE $O/$TAG.pmc_WRITE_SIZE k_paths $O/pmc_$SCENE.json || exit 1
cp $O/pmc_$SCENE.json $R/profiles/pmc_$SCENE.json
cd $R
timeout -k 10 600 python bench.py --scene $SCENE > $O/$TAG.bench.log 2>&1 || { tail -5 $O/$TAG.bench.log; exit 1; }
grep '^{' $O/$TAG.bench.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$TAG.prof -o run --output-format csv -- \
  python $R/bench.py --no-cpu-baseline --scene $SCENE > $O/$TAG.prof.log 2>&1 || { tail -5 $O/$TAG.prof.log; exit 1; }
grep '^{' $O/$TAG.prof.log
python $R/tools/stats.py $O/$TAG.prof
