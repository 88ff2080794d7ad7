#!/bin/bash
# tools/counters.sh for every config (run via gpurun from the repo root):
#   bash tools/counters_all.sh TAG [cfg ...]   -> gpurun_out/TAG_<cfg>.json
# Frames are cut to 256 spp where a full one takes seconds: counters.py records the
# profiled frame's world rays, and bench.py prices the counts per world ray.
set -o pipefail
R=$PWD; O=$R/gpurun_out
TAG=${1:-cnt}; shift
want=" $* "
while read -r tag args; do
  [ -z "$tag" ] && continue
  [ "$want" != "  " ] && [[ "$want" != *" $tag "* ]] && continue
  bash tools/counters.sh ${TAG}_$tag $args > $O/${TAG}_$tag.log 2>&1 || { echo "counters $tag failed"; tail -5 $O/${TAG}_$tag.log; exit 1; }
  echo "$tag: $(python -c "import json; d=json.load(open('$O/${TAG}_$tag.json')); print(d['ms_per_launch_profiled'], 'ms', d.get('valu_lane_utilisation'), 'lanes', d['hbm']['total_bytes'], 'B', d['world_rays_per_launch'], 'rays')")"
done <<'CFG'
s2 --scene s2
s1 --scene s1
s3 --scene s3
s3_metal --scene s3_metal
s4 --scene s4 --spp 256
s5 --scene s5 --spp 256
s2_d100 --scene s2 --divs 100
s4_real --scene s4_real --spp 256
ball --scene ball
random --scene random
CFG
