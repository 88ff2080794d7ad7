set -o pipefail
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullframe.py tests/test_soldier_scene.py tests/test_ref_scenes.py > gpurun_out/r4_bvh_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_bvh_tests.log; [ $rc -eq 0 ] || exit 1
BENCH_ARGS="" bash tools/ab_libs.sh r4bvhc2 opt1:X=0 opt0:SRR_BVH_OPT=0 occ5:SRR_LIB=$L/exp_occ5.so;SRR_PATHS_OCC=5;SRR_BIGBLOCK=0 || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4bvhc4 opt1:X=0 opt0:SRR_BVH_OPT=0 occ5:SRR_LIB=$L/exp_occ5.so;SRR_PATHS_OCC=5;SRR_BIGBLOCK=0 || exit 1
BENCH_ARGS="--scene s4_real --steps 2" bash tools/ab_libs.sh r4bvhc4r opt1:X=0 opt0:SRR_BVH_OPT=0 || exit 1
BENCH_ARGS="--scene s2 --divs 100" bash tools/ab_libs.sh r4bvhd100 opt1:X=0 opt0:SRR_BVH_OPT=0 || exit 1
for o in 0 1; do for a in "--scene s4_real --spp 64" "--spp 64"; do
  SRR_BVH_OPT=$o timeout -k 10 300 python bench.py --no-cpu-baseline --count-visits --steps 1 --warmup 0 $a > gpurun_out/r4_visits_$o$(echo "$a" | tr -c 'a-z0-9' '_').log 2>&1 || exit 1
  echo "opt $o $a: $(grep -o '"visits": {[^}]*}' gpurun_out/r4_visits_$o$(echo "$a" | tr -c 'a-z0-9' '_').log)"
done; done
