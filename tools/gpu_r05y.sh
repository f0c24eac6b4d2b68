#!/bin/bash
# r05y: waves-per-SIMD launch bounds re-checked with non-temporal record traffic (N* Fitch)
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default down6 plain5 plain8 leafy5 subup5 tail5 tail8
