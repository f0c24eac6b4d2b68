#!/bin/bash
# r05ab: non-temporal record loads only in launches of >= 64k waves -- N* and C3 against the
# build before any non-temporal load (r05v)
set -o pipefail
cd "$(dirname "$0")/.."
tools/ab_variants.sh fitch 2 default r05v && tools/ab_variants.sh sankoff 1 default r05v \
  && BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh fitch 2 default r05v \
  && BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh sankoff 2 default r05v
