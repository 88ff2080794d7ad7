#!/bin/bash
# bench the path engine at several occupancy targets: bash tools/occ.sh "2 3 4" [bench.py args...]
OCCS=$1; shift
TAG=$(echo "$@" | tr -c 'a-zA-Z0-9' '_')
for o in $OCCS; do
  SRR_PATHS_OCC=$o timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/occ$o$TAG.log 2>&1 || { echo "occ $o failed"; tail -3 gpurun_out/occ$o$TAG.log; exit 1; }
  echo "occ=$o $* $(python -c "import json; d=json.loads([l for l in open('gpurun_out/occ$o$TAG.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['trace_ms_per_launch'], d['config']['world_rays_per_step'])")"
done
