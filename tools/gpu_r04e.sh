#!/bin/bash
# C3 A/Bs (slots / wide prefetch, Sankoff slots, sub-down), replay variants, FETCH calibration
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default noslots base || exit 4
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh sankoff 1 default noslots || exit 10
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 2 "--sub-down 0" "--sub-down 1" || exit 8
bash tools/replay_variants.sh base rp_e4w5 rp_e8w5 rp_e16w4 || exit 6
bash tools/fetch_calibrate.sh || exit 5
