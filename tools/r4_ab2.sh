set -o pipefail
L=$PWD/simple-raytracing-render_amd
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r4_sg_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r4_sg_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_cfgs.sh r4sg sg:X=0 presg:SRR_LIB=$L/exp_presg.so
# phase timing (diagnostics build) of C2, C4, C4_real, C5
for a in "" "--scene s4 --steps 1" "--scene s4_real --steps 1" "--scene s5 --steps 1 --spp 1024"; do
  SRR_LIB=$L/libsrr_diag.so SRR_PATHS_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline --no-pipeline --warmup 0 --steps 1 $a > gpurun_out/r4_timing_$(echo "x$a" | tr -c 'a-z0-9' '_').log 2>&1 || exit 1
done
grep -h "per wave-iteration\|mixture loop" gpurun_out/r4_timing_*.log
