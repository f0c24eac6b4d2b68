#!/bin/bash
# r05aa: C3 (T2 100k x 30k) Sankoff / Fitch against the build before the non-temporal record
# loads (r05v) and without the Sankoff-side ones (norecnt)
set -o pipefail
cd "$(dirname "$0")/.."
BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh sankoff 2 default r05v norecnt \
  && BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh fitch 2 default r05v
