#!/bin/bash
# frames in flight: bench with two (default) vs one (--no-pipeline), alternating, on C1 / C2 / C4 (run via gpurun)
set -o pipefail
O=gpurun_out
for sc in "--scene s1 --steps 30 --warmup 3" "--scene s2 --steps 6" "--scene s4 --steps 3"; do
  tag=$(echo $sc | cut -c9-10)
  for rep in 1 2; do
    for mode in pipe sync; do
      extra=""; [ $mode = sync ] && extra="--no-pipeline"
      timeout -k 10 300 python bench.py --no-cpu-baseline $sc $extra > $O/pl_${tag}_${mode}_$rep.log 2>&1 || { echo "$sc $mode failed"; tail -3 $O/pl_${tag}_${mode}_$rep.log; exit 1; }
      echo "$tag $mode rep $rep: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"trace_ms_per_launch": [0-9.]*\|"world_rays_per_step": [0-9]*' $O/pl_${tag}_${mode}_$rep.log | tr '\n' ' ')"
    done
  done
done
