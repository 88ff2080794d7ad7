set -o pipefail
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_ring_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_ring_tests.log; [ $rc -eq 0 ] || exit 1
BENCH_ARGS="" bash tools/ab_libs.sh r4ringc2 ring:X=0 noring:SRR_LIB=$L/exp_noring.so || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4ringc1 ring:X=0 noring:SRR_LIB=$L/exp_noring.so || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4ringc4 ring:X=0 noring:SRR_LIB=$L/exp_noring.so || exit 1
