set -o pipefail
# mesh-free path kernel variant (no BVH4 walk, no LDS stacks / node cache) at 4 (nm4) or 5 (nm5) waves per SIMD, vs HEAD
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_nm4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_nm4_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_nm4_tests.log; [ $rc -eq 0 ] || exit 1
SRR_LIB=$L/exp_nm5.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_ref_scenes.py > gpurun_out/r4_nm5_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_nm5_tests.log; [ $rc -eq 0 ] || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4nmc1 head:X=0 nm4:SRR_LIB=$L/exp_nm4.so nm5:SRR_LIB=$L/exp_nm5.so t1:SRR_LIB=$L/exp_tops1.so || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4nmc1b head:X=0 nm4:SRR_LIB=$L/exp_nm4.so nm5:SRR_LIB=$L/exp_nm5.so t1:SRR_LIB=$L/exp_tops1.so
