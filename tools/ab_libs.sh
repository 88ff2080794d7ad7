#!/bin/bash
# A/B of alternative builds / env knobs on one bench config (run via gpurun):
#   tools/ab_libs.sh TAG "name:ENV=..;.." ...   each entry: a label, then space-free env assignments
#   separated by ';' (SRR_LIB=... selects a library).  Two alternating passes.
TAG=$1; shift
O=gpurun_out
for rep in 1 2; do
  for e in "$@"; do
    name=${e%%:*}; envs=${e#*:}
    env ${envs//;/ } timeout -k 10 200 python bench.py --steps 4 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/$TAG.$name.$rep.log 2>&1 || { echo "$name failed"; tail -3 $O/$TAG.$name.$rep.log; exit 1; }
    echo "$name rep $rep: $(grep -o '"value": [0-9.]*' $O/$TAG.$name.$rep.log) $(grep -o '"world_rays_per_step": [0-9]*' $O/$TAG.$name.$rep.log)"
  done
done
