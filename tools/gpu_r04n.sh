#!/bin/bash
# C3 schedule parameters (runtime options only): narrow-band width, pre-order group size
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 2 "--narrow 16" "--narrow 32" "--narrow 64" "--group 65536" "--group 16384" "--group-levels 3" || exit 2
