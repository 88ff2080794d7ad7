#!/bin/bash
# C4 / C5 at 3 vs 4 waves per SIMD (256-lane blocks; exp_occ.so = -DSRR_OCC_VARIANTS): do the
# ALLFAM / MEDIA variants' register spills cost more than the latency a 4th wave hides?
set -o pipefail
L=$PWD/simple-raytracing-render_amd
for sc in "--scene s4 --steps 2" "--scene s5 --spp 512 --steps 2"; do
  BENCH_ARGS="$sc" bash tools/ab_libs.sh occ$(echo $sc | cut -c9-10) \
    "occ4:SRR_LIB=$L/exp_occ.so;SRR_BIGBLOCK=0" "occ5:SRR_LIB=$L/exp_occ.so;SRR_PATHS_OCC=5" "occ6:SRR_LIB=$L/exp_occ.so;SRR_PATHS_OCC=6" || exit 1
done
