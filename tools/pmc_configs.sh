#!/bin/bash
# Measured HBM traffic (FETCH_SIZE / WRITE_SIZE passes, one counter per run) of
# k_paths for every config stand-in -> profiles/pmc_<scene>[_d<divs>].json, which
# bench.py reports as roofline.traffic.  Run via gpurun from the repo root.
set -o pipefail
R=$PWD
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for args in "--scene s1" "--scene s2" "--scene s3" "--scene s3_metal" "--scene s4" "--scene s5" "--scene s2 --divs 100" "--scene s4_real"; do
  tag=$(echo $args | sed 's/--scene //; s/ --divs /_d/')
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $O/pmcc_${tag}_$c -o run -- \
      python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline $args > $O/pmcc_${tag}_$c.log 2>&1 \
      || { echo "pmc $c $args failed"; tail -5 $O/pmcc_${tag}_$c.log; exit 1; }
  done
  python $R/tools/pmc_traffic.py $O/pmcc_${tag}_FETCH_SIZE $O/pmcc_${tag}_WRITE_SIZE k_paths $R/profiles/pmc_$tag.json $O/pmcc_${tag}_FETCH_SIZE.log || exit 1
  cp $R/profiles/pmc_$tag.json $O/
  echo "$tag $(python -c "import json; print(json.load(open('$R/profiles/pmc_$tag.json'))['hbm_bytes_per_launch'])")"
done
