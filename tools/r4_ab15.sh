set -o pipefail
# product build (no scratch objects: light triangle read in place, diffuse set-up selected by value,
# both prepared BSDF terms always written) vs the previous HEAD (exp_head.so)
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_sf_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_sf_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4sf new:X=0 head:SRR_LIB=$L/exp_head.so || exit 1
BENCH_ARGS="--scene s3 --steps 2" bash tools/ab_libs.sh r4sfc3 new:X=0 head:SRR_LIB=$L/exp_head.so || exit 1
BENCH_ARGS="--scene s4_real --steps 1" bash tools/ab_libs.sh r4sfc4r new:X=0 head:SRR_LIB=$L/exp_head.so
