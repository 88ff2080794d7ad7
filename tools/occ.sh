#!/bin/bash
# bench the path engine at several occupancy targets
for o in "$@"; do
  SRR_PATHS_OCC=$o timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/occ$o.log 2>&1 || { echo "occ $o failed"; tail -3 gpurun_out/occ$o.log; exit 1; }
  echo "occ=$o $(python -c "import json; d=json.loads([l for l in open('gpurun_out/occ$o.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['trace_ms_per_launch'])")"
done
