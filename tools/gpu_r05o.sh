#!/bin/bash
# r05o: replay parity with non-temporal row stores; N* A/B of non-temporal post-order / record stores
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_replay.py tests/test_gpu_reroot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05o_tests.log 2>&1 \
  || { echo "REPLAY TESTS FAILED"; tail -60 gpurun_out/r05o_tests.log; exit 1; }
tail -1 gpurun_out/r05o_tests.log
tools/ab_variants.sh fitch 2 default upnt recnt && tools/ab_variants.sh sankoff 1 default upnt recnt
