#!/bin/bash
# Bench line for every BASELINE config stand-in on one GPU (run via gpurun from the repo root).
set -o pipefail
for sc in s1 s3 s3_metal s4 s5; do
  timeout -k 10 600 python bench.py --scene $sc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cfg_$sc.log 2>&1 || { echo "$sc failed"; tail -3 gpurun_out/cfg_$sc.log; exit 1; }
  grep '^{' gpurun_out/cfg_$sc.log
done
