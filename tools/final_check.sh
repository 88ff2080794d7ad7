#!/bin/bash
# End-of-round check of the committed build on one GPU (run via gpurun from the repo root):
# GPU tests, smoke(), the default bench line (with cpu_baseline), and a rocprofv3 kernel-trace
# summary of the same bench command.   bash tools/final_check.sh TAG
set -o pipefail
TAG=${1:-final}
R=$PWD; O=$R/gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/$TAG.tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 $O/$TAG.tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/$TAG.smoke.log 2>&1 || { tail -5 $O/$TAG.smoke.log; exit 1; }
tail -1 $O/$TAG.smoke.log
timeout -k 10 600 python bench.py > $O/$TAG.bench.log 2>&1 || { tail -5 $O/$TAG.bench.log; exit 1; }
grep '^{' $O/$TAG.bench.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$TAG.prof -o run --output-format csv -- \
  python $R/bench.py --no-cpu-baseline > $O/$TAG.prof.log 2>&1 || { tail -5 $O/$TAG.prof.log; exit 1; }
python $R/tools/stats.py $O/$TAG.prof
