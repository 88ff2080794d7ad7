O=gpurun_out
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_paths_match_reference" "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame" "tests/test_gpu_parity.py::test_larger_renders_match_oracle_on_sampled_pixels" > $O/lq.tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/lq.tests.log
BENCH_ARGS="" bash tools/ab_libs.sh lqc2 lq0:SRR_LIB=$L/exp_lq0.so lq1:X=0
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh lqc4 lq0:SRR_LIB=$L/exp_lq0.so lq1:X=0
BENCH_ARGS="--scene s4_real --steps 2" bash tools/ab_libs.sh lqc4r lq0:SRR_LIB=$L/exp_lq0.so lq1:X=0
