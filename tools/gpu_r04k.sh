#!/bin/bash
# The round's evidence on the final build: N* Fitch and Sankoff profiles (stats + FETCH / WRITE /
# SQ), C3 / C3 Sankoff / C2 traces, replay PMC
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04k.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04k.log; exit 9; }
tail -1 gpurun_out/gputests_r04k.log
bash tools/profile_fitch.sh r04 || exit 2
bash tools/profile_fitch.sh r04_sankoff --mode sankoff || exit 3
bash tools/trace_stats.sh r04_c3 --tree sars-like --leaves 100000 --steps 5 --warmup 2 || exit 4
bash tools/trace_stats.sh r04_c3_sankoff --tree sars-like --leaves 100000 --mode sankoff --steps 5 --warmup 2 || exit 5
bash tools/trace_stats.sh r04_c2 --leaves 4096 --sites 15000 --steps 10 --warmup 3 || exit 6
bash tools/profile_replay.sh r04 || exit 7
