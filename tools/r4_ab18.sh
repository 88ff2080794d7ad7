set -o pipefail
# coop_mixture's deep-tries threshold (failed attempts after which a path takes every free lane): 32 (default) vs 16 vs 64
BENCH_ARGS="" bash tools/ab_libs.sh r4dtc2 dt32:X=0 dt16:SRR_DEEP_TRIES=16 dt64:SRR_DEEP_TRIES=64 || exit 1
BENCH_ARGS="--scene s4 --steps 2" bash tools/ab_libs.sh r4dtc4 dt32:X=0 dt16:SRR_DEEP_TRIES=16 dt64:SRR_DEEP_TRIES=64 || exit 1
BENCH_ARGS="--scene s1 --steps 30 --warmup 3" bash tools/ab_libs.sh r4dtc1 dt32:X=0 dt16:SRR_DEEP_TRIES=16 dt64:SRR_DEEP_TRIES=64
