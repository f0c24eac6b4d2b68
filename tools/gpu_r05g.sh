#!/bin/bash
# r05g: C4 rank share and N* on one box: this build vs the round-3 and round-4 final builds.
set -o pipefail
cd "$(dirname "$0")/.."
BENCH_ARGS="--leaves 8000000 --sites 3750" tools/ab_variants.sh fitch 2 default rev_r03 rev_r04 && \
tools/ab_variants.sh fitch 2 default rev_r03 rev_r04
