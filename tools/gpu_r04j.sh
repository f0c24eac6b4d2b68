#!/bin/bash
# Replay: double-buffered tile copy-in (default) vs single buffer (nodb); replay tests
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04j.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04j.log; exit 3; }
tail -1 gpurun_out/gputests_r04j.log
bash tools/replay_variants.sh base nodb base nodb || exit 6
