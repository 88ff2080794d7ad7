set -o pipefail
# the record column address re-derived at each use (exp_slot.so) vs the product build
L=$PWD/simple-raytracing-render_amd
SRR_LIB=$L/exp_slot.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_slot_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_slot_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4sl head:X=0 slot:SRR_LIB=$L/exp_slot.so || exit 1
BENCH_ARGS="--scene s3 --steps 2" bash tools/ab_libs.sh r4slc3 head:X=0 slot:SRR_LIB=$L/exp_slot.so || exit 1
BENCH_ARGS="--scene s4_real --steps 1" bash tools/ab_libs.sh r4slc4r head:X=0 slot:SRR_LIB=$L/exp_slot.so
