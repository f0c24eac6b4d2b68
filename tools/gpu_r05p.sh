#!/bin/bash
# r05p: full GPU suite on the non-temporal-store build; A/B of non-temporal leaf loads / mask stores
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r05p.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_r05p.log; exit 1; }
tail -1 gpurun_out/gputests_r05p.log
tools/ab_variants.sh fitch 2 default leafup leafdown masknt && tools/ab_variants.sh sankoff 1 default leafup leafdown masknt
