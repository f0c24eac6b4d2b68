#!/bin/bash
# Compact complex lanes: core Fitch parity tests, then N* / C3 A/B against the 16-plane format
# (build_var/$VAR):  tools/gpu_r06cx.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_fitch.py tests/test_gpu_group.py tests/test_gpu_narrow.py tests/test_gpu_cluster.py tests/test_gpu_block.py tests/test_gpu_graph.py} > gpurun_out/${tag}_tests.log 2>&1 || { echo TESTS FAILED; grep -E "FAILED|Error|error" gpurun_out/${tag}_tests.log | head -20; tail -5 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
[ -n "${NOAB:-}" ] && exit 0
bash tools/ab_variants.sh fitch ${REPS:-2} default ${VAR:-cx0} || exit 2
BENCH_ARGS="--tree sars-like --leaves 100000" bash tools/ab_variants.sh fitch 2 default ${VAR:-cx0} || exit 3
[ -n "${SK:-}" ] && { bash tools/ab_variants.sh sankoff 1 default ${VAR:-cx0} || exit 4; }
