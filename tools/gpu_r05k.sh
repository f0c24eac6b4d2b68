#!/bin/bash
# r05k: early record reservation -- full GPU parity suite, then N* A/B of the reservation size
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r05k.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/gputests_r05k.log; exit 1; }
tail -2 gpurun_out/gputests_r05k.log
tools/ab_variants.sh fitch 2 default reserve0 reserve4 reserve16 && tools/ab_variants.sh sankoff 1 default reserve0
