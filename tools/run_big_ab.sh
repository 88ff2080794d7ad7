O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu "tests/test_gpu_parity.py::test_paths_match_reference" "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame" tests/test_mixture_cap.py "tests/test_gpu_parity.py::test_larger_renders_match_oracle_on_sampled_pixels" > $O/big.tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/big.tests.log
BENCH_ARGS="" bash tools/ab_libs.sh bigc2 small:SRR_BIGBLOCK=0 big:X=0 bigq:SRR_CBVH=1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh bigc4 small:SRR_BIGBLOCK=0 big:X=0
BENCH_ARGS="--divs 100 --steps 2" bash tools/ab_libs.sh bigd100 small:SRR_BIGBLOCK=0 big:X=0 bigq:SRR_CBVH=1
