#!/bin/bash
# Bench line for every BASELINE config stand-in on one GPU (run via gpurun from the repo root),
# plus C2 with the reference's as-shipped 640,000-triangle teapot (teapot.h:77) and the reference's
# as-shipped default run (ball_scenes) and random_scene at its globals 1000x1000x50.  Every line
# carries cpu_baseline: the reference's own code on the host CPUs available to the job.
#   bash tools/configs.sh [TAG]     -> gpurun_out/TAG_<cfg>.log, TAG.jsonl
set -o pipefail
TAG=${1:-cfg}
: > gpurun_out/$TAG.jsonl
for args in "--scene s1 --steps 30 --warmup 3" "--scene s2" "--scene s3" "--scene s3_metal" "--scene s4" "--scene s5" \
            "--scene s2 --divs 100" "--scene s4_real" "--scene ball --steps 10 --warmup 2" "--scene random --steps 10 --warmup 2"; do
  tag=$(echo $args | tr -c 'a-z0-9' '_')
  case "$args" in *--steps*) st="";; *) st="--steps 2 --warmup 1";; esac
  timeout -k 10 600 python bench.py $args $st > gpurun_out/${TAG}_$tag.log 2>&1 || { echo "$args failed"; tail -3 gpurun_out/${TAG}_$tag.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_$tag.log | tee -a gpurun_out/$TAG.jsonl | cut -c1-160
done
