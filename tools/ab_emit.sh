#!/bin/bash
# Post-order emission A/B on the GPU box: its equality tests, then N* Fitch with it off / on.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fitch.py -k "up_emit or all_present or synthetic" -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_emit_tests.log 2>&1 \
  || { echo "TESTS FAILED"; tail -40 gpurun_out/ab_emit_tests.log; exit 1; }
tail -1 gpurun_out/ab_emit_tests.log
for v in 0 1 0 1; do
  timeout -k 10 300 python bench.py --no-cpu --with none --steps 10 --warmup 3 --up-emit $v > gpurun_out/ab_emit_$v.json 2> gpurun_out/ab_emit_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_emit_$v.err; exit 2; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_emit_$v.json'));r=d['roofline'];print('emit $v', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
done
