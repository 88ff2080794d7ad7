set -o pipefail
# bounce records of the first bounces in LDS for mesh-free scenes (exp_ldsrec.so) vs HEAD
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_ldsrec.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_ldsrec_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_ldsrec_tests.log; [ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4lrc1 head:X=0 ldsrec:SRR_LIB=$L/exp_ldsrec.so || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4lrc4 head:X=0 ldsrec:SRR_LIB=$L/exp_ldsrec.so || exit 1
BENCH_ARGS="--scene s5 --steps 1" bash tools/ab_libs.sh r4lrc5 head:X=0 ldsrec:SRR_LIB=$L/exp_ldsrec.so || exit 1
BENCH_ARGS="" bash tools/ab_libs.sh r4lrc2 head:X=0 ldsrec:SRR_LIB=$L/exp_ldsrec.so
