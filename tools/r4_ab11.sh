set -o pipefail
# packed slab arithmetic in mesh_hit4 (pk), + wave ray/cap totals in SGPRs (pksg) or LDS (pklds), vs HEAD
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_pksg.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_pk_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_pk_tests.log; [ $rc -eq 0 ] || exit 1
SRR_LIB=$L/exp_pklds.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fullframe.py tests/test_mixture_cap.py tests/test_gpu_parity.py > gpurun_out/r4_pklds_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_pklds_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4pk head:X=0 pk:SRR_LIB=$L/exp_pkslab.so pksg:SRR_LIB=$L/exp_pksg.so pklds:SRR_LIB=$L/exp_pklds.so || exit 1
BENCH_ARGS="--scene s4_real --steps 1" bash tools/ab_libs.sh r4pkc4r head:X=0 pk:SRR_LIB=$L/exp_pkslab.so pksg:SRR_LIB=$L/exp_pksg.so
