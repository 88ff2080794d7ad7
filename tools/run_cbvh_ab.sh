O=gpurun_out
SRR_CBVH=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_paths_match_reference" "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame[default]" "tests/test_gpu_parity.py::test_larger_renders_match_oracle_on_sampled_pixels" > $O/cb.tests.log 2>&1; echo "cbvh tests rc=$?"; tail -2 $O/cb.tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame[default]" > $O/cb.tests0.log 2>&1; echo "sobol fullframe rc=$?"
BENCH_ARGS="" bash tools/ab_libs.sh cbc2 base:X=0 cbvh:SRR_CBVH=1
BENCH_ARGS="--divs 100 --steps 2" bash tools/ab_libs.sh cbd100 quad:X=0 lane:SRR_QUAD=0 lanecbvh:SRR_QUAD=0;SRR_CBVH=1
L=$PWD/simple-raytracing-render_amd
BENCH_ARGS="" bash tools/ab_libs.sh noslp base:X=0 noslp:SRR_LIB=$L/exp_noslp.so
