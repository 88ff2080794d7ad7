#!/bin/bash
# kernel-trace profile of one bench step: tools/prof.sh TAG [bench args]
TAG=$1; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG.prof -o run --output-format csv -- python $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/$TAG.prof.log 2>&1 || { tail -5 $R/gpurun_out/$TAG.prof.log; exit 1; }
grep metric $R/gpurun_out/$TAG.prof.log | cut -c1-300
