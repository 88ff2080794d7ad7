#!/bin/bash
# Bench line for every BASELINE config stand-in on one GPU (run via gpurun from the repo root),
# plus C2 with the reference's as-shipped 640,000-triangle teapot (teapot.h:77).
set -o pipefail
for args in "--scene s1 --steps 30 --warmup 3" "--scene s2" "--scene s3" "--scene s3_metal" "--scene s4" "--scene s5" "--scene s2 --divs 100" "--scene s4_real"; do
  tag=$(echo $args | tr -c 'a-z0-9' '_')
  case "$args" in *--steps*) st="";; *) st="--steps 2 --warmup 1";; esac
  timeout -k 10 600 python bench.py $args $st --no-cpu-baseline > gpurun_out/cfg_$tag.log 2>&1 || { echo "$args failed"; tail -3 gpurun_out/cfg_$tag.log; exit 1; }
  grep '^{' gpurun_out/cfg_$tag.log
done
