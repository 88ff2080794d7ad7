#!/bin/bash
# C5 HBM traffic per world ray at 4 waves/SIMD (7 spilled VGPRs) vs 3 waves/SIMD (no spills):
# does register spilling (scratch beyond L2) carry C5's traffic?  (run via gpurun; exp_occ.so
# = -DSRR_OCC_VARIANTS)
set -o pipefail
R=$PWD; O=$R/gpurun_out; L=$R/simple-raytracing-render_amd/exp_occ.so
cd /tmp && export TMPDIR=/tmp
for occ in 4 3; do
  for c in FETCH_SIZE WRITE_SIZE; do
    env SRR_LIB=$L SRR_PATHS_OCC=$occ SRR_BIGBLOCK=0 timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pocc${occ}_$c -o run -- \
      python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --scene s5 --spp 256 > $O/pocc${occ}_$c.log 2>&1 || { echo "occ $occ $c failed"; tail -3 $O/pocc${occ}_$c.log; exit 1; }
  done
  python $R/tools/pmc_traffic.py $O/pocc${occ}_FETCH_SIZE $O/pocc${occ}_WRITE_SIZE k_paths $O/pocc${occ}.json || exit 1
  rays=$(grep -o '"world_rays_per_step": [0-9]*' $O/pocc${occ}_FETCH_SIZE.log | grep -o '[0-9]*$')
  python -c "import json; d=json.load(open('$O/pocc${occ}.json')); print('occ $occ: read %.1f write %.1f B per world ray' % (d['read_bytes_per_launch']/$rays, d['write_bytes_per_launch']/$rays))"
done
