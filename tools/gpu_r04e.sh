#!/bin/bash
# C3 A/Bs: current (slots + plain) vs the S / other split child sets (no spilling grouped kernels)
# vs no slots vs round-3-era base; Sankoff likewise; sub-down; replay variants
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default split noslots base || exit 4
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh sankoff 1 default split noslots || exit 10
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_args.sh 1 "--sub-down 0" "--sub-down 1" || exit 8
bash tools/replay_variants.sh base rp_e4w5 rp_e8w5 rp_e16w4 || exit 6
