#!/bin/bash
# A/B of the default build against LIB on C2, C4, the 640k teapot and C4_real (run via gpurun)
#   bash tools/ab_scenes.sh TAG LIB
set -o pipefail
L=$PWD/simple-raytracing-render_amd
for sc in "--scene s4 --steps 2" "--scene s2 --divs 100 --steps 3" "--scene s4_real --steps 2" ""; do
  BENCH_ARGS="$sc" bash tools/ab_libs.sh $1$(echo $sc | tr -dc 'a-z0-9' | cut -c1-12) "base:X=0" "exp:SRR_LIB=$L/$2" || exit 1
done
