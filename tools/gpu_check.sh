#!/bin/bash
# usage: tools/gpu_check.sh TAG  -- GPU tests, bench, kernel-trace profile (run via gpurun)
TAG=${1:-run}
R=$PWD
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG.tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/$TAG.tests.log
tail -2 gpurun_out/$TAG.tests.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || exit 1
grep metric gpurun_out/$TAG.bench.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG.prof -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $R/gpurun_out/$TAG.prof.log 2>&1 || exit 1
cut -d, -f1-4 $R/gpurun_out/$TAG.prof/run_kernel_stats.csv | cut -c1-160
