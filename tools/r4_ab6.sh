set -o pipefail
L=$PWD/simple-raytracing-render_amd
BENCH_ARGS="--scene s4_real --steps 2" bash tools/ab_libs.sh r4ldsc4r base:X=0 noring:SRR_LIB=$L/exp_noring.so k6:SRR_LIB=$L/exp_k6.so || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4ldsc4 base:X=0 noring:SRR_LIB=$L/exp_noring.so k6:SRR_LIB=$L/exp_k6.so || exit 1
BENCH_ARGS="" bash tools/ab_libs.sh r4ldsc2 base:X=0 noring:SRR_LIB=$L/exp_noring.so k6:SRR_LIB=$L/exp_k6.so || exit 1
