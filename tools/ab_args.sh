#!/bin/bash
# A/B of library builds on chosen bench arguments (run via gpurun from the repo root):
#   tools/ab_args.sh TAG "ARGS1" "ARGS2" -- LIB1 LIB2 ...
TAG=$1; shift
ARGS=()
while [ "$1" != "--" ]; do ARGS+=("$1"); shift; done
shift
for a in "${ARGS[@]}"; do
  for lib in "$@"; do
    SRR_LIB=$PWD/$lib timeout -k 10 300 python bench.py $a --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG.bench.log 2>&1 || { echo "bench failed for $lib $a"; tail -5 gpurun_out/$TAG.bench.log; exit 1; }
    echo "$a | $lib $(python -c "import json; d=json.loads([l for l in open('gpurun_out/$TAG.bench.log') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['trace_ms_per_launch'])")"
  done
done
