#!/bin/bash
# child-set formulations: branch-free for every child (default) vs branchy (prebf) vs a uniform
# S-subtree / other split (split; splitl: the leafy kernel too; splitsk5: Sankoff at 5 waves)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/ab_variants.sh fitch 2 default prebf split splitl || exit 2
bash tools/ab_variants.sh sankoff 2 default prebf split splitsk5 || exit 3
