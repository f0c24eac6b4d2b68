#!/bin/bash
# Tests after the plain threshold + Sankoff plain kernel + replay double buffer; A/B plain on/off
# (N* Fitch, Sankoff); C3 vs no slots; replay DB vs single buffer
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_gpu_sankoff.py tests/test_gpu_fitch.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py tests/test_gpu_replay.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04i.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04i.log; exit 3; }
tail -1 gpurun_out/gputests_r04i.log
bash tools/replay_variants.sh base nodb base nodb || exit 8
bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 4
BENCH_ARGS="--mode sankoff" bash tools/ab_args.sh 1 "--plain-up 0" "--plain-up 1" || exit 5
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default noslots || exit 6
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh sankoff 1 default noslots || exit 7
