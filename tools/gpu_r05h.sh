#!/bin/bash
# r05h: polytomy / group / narrow parity, then C3 (T2 100k x 30k) A/B of the wide-node fetch depth.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_narrow.py tests/test_gpu_group.py tests/test_gpu_fitch.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/r05h_tests.log; exit 1; }
tail -1 gpurun_out/r05h_tests.log
BENCH_ARGS="--tree sars-like --leaves 100000" tools/ab_variants.sh fitch 3 default wide2
