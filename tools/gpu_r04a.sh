set -o pipefail
bash tools/gpu_round_check.sh r04a || exit 1
bash tools/ab_variants.sh fitch 2 default occ3 occ2
