#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/gpu_round_check.sh r04c || exit 1
bash tools/ab_variants.sh fitch 2 default occ3 occ2 || exit 2
bash tools/gpu_r04b.sh r04c || exit 3
