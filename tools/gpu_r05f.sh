#!/bin/bash
# r05f: replay parity (the final DFS build), then the C4 rank share (8M leaves x 3750 sites)
# attribution: plain split on / off / higher threshold.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay_deep.py tests/test_gpu_replay.py tests/test_gpu_reroot.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || { echo "REPLAY TESTS FAILED"; tail -40 gpurun_out/r05f_tests.log; exit 1; }
tail -1 gpurun_out/r05f_tests.log
BENCH_ARGS="--leaves 8000000 --sites 3750" tools/ab_args.sh 2 "--plain-up 1" "--plain-up 0" "--plain-up 262144"
