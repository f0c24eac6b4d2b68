#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sankoff.py tests/test_gpu_fitch.py tests/test_gpu_group.py tests/test_gpu_narrow.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r04d2.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests_r04d2.log; exit 3; }
tail -1 gpurun_out/gputests_r04d2.log
bash tools/ab_variants.sh sankoff 2 default noslots || exit 9
bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 11
bash tools/ab_variants.sh fitch 2 default plain5 || exit 12
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default noslots base || exit 4
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh sankoff 1 default noslots || exit 10
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 2 "--sub-down 0" "--sub-down 1" || exit 8
bash tools/replay_variants.sh base rp_e4w5 rp_e8w5 rp_e16w4 || exit 6
