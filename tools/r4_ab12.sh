set -o pipefail
# top-level world objects as one 48-B DTop (object + first two transforms) from LDS (t1), or
# from global memory with scalar loads prefetched one object ahead (t2), vs HEAD
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_tops1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_t1_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_t1_tests.log; [ $rc -eq 0 ] || exit 1
SRR_LIB=$L/exp_tops2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullframe.py tests/test_gpu_parity.py > gpurun_out/r4_t2_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_t2_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4t head:X=0 t1:SRR_LIB=$L/exp_tops1.so t2:SRR_LIB=$L/exp_tops2.so || exit 1
BENCH_ARGS="--scene s3 --steps 2" bash tools/ab_libs.sh r4tc3 head:X=0 t1:SRR_LIB=$L/exp_tops1.so t2:SRR_LIB=$L/exp_tops2.so
