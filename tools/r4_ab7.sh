set -o pipefail
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullframe.py tests/test_soldier_scene.py tests/test_ref_scenes.py > gpurun_out/r4_run_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_run_tests.log; [ $rc -eq 0 ] || exit 1
E="run:X=0 prev:SRR_LIB=$L/exp_prev.so noring:SRR_LIB=$L/exp_noring.so k6:SRR_LIB=$L/exp_k6.so k6noring:SRR_LIB=$L/exp_k6noring.so"
BENCH_ARGS="" bash tools/ab_libs.sh r4l2c2 $E || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4l2c1 $E || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4l2c4 $E || exit 1
BENCH_ARGS="--scene s4_real --steps 2" bash tools/ab_libs.sh r4l2c4r $E || exit 1
