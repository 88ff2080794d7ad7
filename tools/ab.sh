#!/bin/bash
# A/B bench variants on one box: tools/ab.sh TAG "ENV1" "ENV2" ...
TAG=$1; shift
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$TAG.tests.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/$TAG.tests.log
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || { echo "bench failed for $v"; tail -5 gpurun_out/$TAG.bench.log; exit 1; }
  echo "$v $(python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/$TAG.bench.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['trace_ms_per_launch'])")"
done
