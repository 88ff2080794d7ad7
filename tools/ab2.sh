#!/bin/bash
# A/B bench of library builds on one box: tools/ab2.sh TAG LIB1 LIB2 ... (paths relative to repo root)
TAG=$1; shift
for lib in "$@"; do
  SRR_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || { echo "bench failed for $lib"; tail -5 gpurun_out/$TAG.bench.log; exit 1; }
  echo "$lib $(python -c "import json; d=json.loads([l for l in open('gpurun_out/$TAG.bench.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['trace_ms_per_launch'])")"
done
