#!/bin/bash
# r05u: per-wave record slots -- full GPU suite, then N* A/B of the slot size (0 = shards only)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r05u.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_r05u.log; exit 1; }
tail -1 gpurun_out/gputests_r05u.log
tools/ab_variants.sh fitch 2 default noslots slots16 slots64 && tools/ab_variants.sh sankoff 1 default noslots
