set -o pipefail
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_light_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_light_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4light new:X=0 prev:SRR_LIB=$L/exp_prev.so || exit 1
BENCH_ARGS="--scene s4_real --steps 2" bash tools/ab_libs.sh r4lightc4r new:X=0 prev:SRR_LIB=$L/exp_prev.so || exit 1
