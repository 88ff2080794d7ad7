#!/bin/bash
# Phase and material-family timing of k_paths (diagnostics build, SRR_PATHS_TIMING=1) for
# several configs (run via gpurun from the repo root):  bash tools/phases.sh TAG [configs...]
# configs: c1 c2 c3 c3m c4 c5 c4r d100 ball random (default: c2 c3 c4 c5 c4r)
set -o pipefail
TAG=${1:-ph}; shift
L=$PWD/simple-raytracing-render_amd
declare -A ARGS=([c1]="--scene s1 --steps 3" [c2]="" [c3]="--scene s3" [c3m]="--scene s3_metal" [c4]="--scene s4"
                 [c5]="--scene s5 --spp 1024" [c4r]="--scene s4_real" [d100]="--scene s2 --divs 100"
                 [ball]="--scene ball --steps 3" [random]="--scene random --steps 3")
for c in ${@:-c2 c3 c4 c5 c4r}; do
  SRR_LIB=$L/libsrr_diag.so SRR_PATHS_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline \
    --warmup 0 --steps 1 ${ARGS[$c]} > gpurun_out/$TAG.$c.log 2>&1 || { echo "$c failed"; tail -3 gpurun_out/$TAG.$c.log; exit 1; }
  echo "== $c"; grep -h "per wave-iteration\|mixture loop\|families:\|  mesh\|  beckmann" gpurun_out/$TAG.$c.log | tail -7
done
