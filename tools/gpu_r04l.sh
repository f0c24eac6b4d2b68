#!/bin/bash
# Final build: plain post-order prefixes on / off (N* Fitch, N* Sankoff, C3)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 2
BENCH_ARGS="--mode sankoff" bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 3
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 2 "--plain-up 0" "--plain-up 1" || exit 4
