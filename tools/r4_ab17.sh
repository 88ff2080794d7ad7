set -o pipefail
# top-level boxes announced by an OBJ_BOUND that lets the wave skip their 6 rects (exp_bnd.so) vs the product build
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_bnd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_bnd_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_bnd_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4bn head:X=0 bnd:SRR_LIB=$L/exp_bnd.so || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4bnc1b head:X=0 bnd:SRR_LIB=$L/exp_bnd.so
