#!/bin/bash
# r05f: C4 rank share (8M leaves x 3750 sites) attribution: plain split on / off / higher
# threshold, leaf-parent pairs on / off; N* beside it.
set -o pipefail
cd "$(dirname "$0")/.."
export BENCH_ARGS="--leaves 8000000 --sites 3750"
tools/ab_args.sh 2 "--plain-up 1" "--plain-up 0" "--plain-up 262144" && \
tools/ab_variants.sh fitch 1 default nopairs
