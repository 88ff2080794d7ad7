#!/bin/bash
# A/B bench of environment settings on one box: tools/ab_env.sh TAG "ENV=.." "ENV=.." ...  ("-" = none)
TAG=$1; shift
for v in "$@"; do
  [ "$v" = "-" ] && v="SRR_AB_NONE=1"
  env $v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || { echo "bench failed for $v"; tail -5 gpurun_out/$TAG.bench.log; exit 1; }
  echo "$v $(python -c "import json; d=json.loads([l for l in open('gpurun_out/$TAG.bench.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['trace_ms_per_launch'])")"
done
