#!/bin/bash
# r05r: non-temporal compact finals (pre-order) A/B
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default finalnt && tools/ab_variants.sh sankoff 2 default finalnt
