set -o pipefail
bash tools/ab_cfgs.sh r4wg lds:X=0 global:SRR_WORLD_GLOBAL=1 || exit 1
