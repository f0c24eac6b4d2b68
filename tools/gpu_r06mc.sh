#!/bin/bash
# Cluster-count band rule (PM_CL_MAX_CLUSTERS) A/B on the C4 (T2) share and C3
set -o pipefail
cd "$(dirname "$0")/.."
PM_CL_DEBUG=1 timeout -k 10 300 python bench.py --no-cpu --with none --steps 3 --warmup 1 --tree sars-like --leaves 100000 > gpurun_out/mc_dbg3.json 2> gpurun_out/mc_dbg3.err || exit 2
grep "^band" gpurun_out/mc_dbg3.err | head -40
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default ${VARS:-mc16384 mc32768} || exit 5
BENCH_ARGS="--tree sars-like --leaves 8000000 --sites 3750" bash tools/ab_variants.sh fitch 1 default ${VARS:-mc16384 mc32768} || exit 3
