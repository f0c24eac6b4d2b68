#!/bin/bash
# r05x: full GPU suite on the non-temporal set-record-load build; A/B of more non-temporal loads
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r05x.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_r05x.log; exit 1; }
tail -1 gpurun_out/gputests_r05x.log
tools/ab_variants.sh fitch 2 default recnt2 pfnt && tools/ab_variants.sh sankoff 2 default recnt2 pfnt \
  && BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh fitch 1 default recnt2 pfnt
