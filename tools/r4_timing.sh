set -o pipefail
L=$PWD/simple-raytracing-render_amd
for a in "--scene s1 --steps 3" "--steps 1" "--scene s3 --steps 1"; do
  t=$(echo "x$a" | tr -c 'a-z0-9' '_')
  SRR_LIB=$L/libsrr_diag.so SRR_PATHS_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline --warmup 1 $a > gpurun_out/r4t2_$t.log 2>&1 || exit 1
  echo "$a"; grep -h "per wave-iteration\|mixture loop" gpurun_out/r4t2_$t.log | tail -2
done
SRR_WAVE_TIMES=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline --warmup 1 --steps 1 --scene s1 > gpurun_out/r4t2_wavetimes_s1.log 2>&1 || exit 1
grep -h "wave exits" gpurun_out/r4t2_wavetimes_s1.log | tail -2
