#!/bin/bash
# r05e: every GPU test; N* A/B leaf-parent pairs (default) vs none; replay DFS variants + PMC.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1 \
  || { echo "GPU TESTS FAILED"; tail -60 gpurun_out/r05e_tests.log; exit 1; }
tail -1 gpurun_out/r05e_tests.log
tools/ab_variants.sh fitch 2 default nopairs && tools/ab_variants.sh sankoff 1 default nopairs && \
tools/replay_variants.sh base dfstm dfsne dfslite && tools/profile_replay_dfs.sh base
