#!/bin/bash
# Fitch GPU tests (fast subset) + N* Fitch with (default build)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_fitch.py tests/test_gpu_narrow.py tests/test_gpu_graph.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_quick.log 2>&1 || { echo TESTS FAILED; tail -40 gpurun_out/gputests_quick.log; exit 1; }
tail -1 gpurun_out/gputests_quick.log
for v in ${VARIANTS:-default}; do
  a=""
  timeout -k 10 200 python bench.py --no-cpu --with none --steps 10 --warmup 3 $a $BENCH_ARGS > gpurun_out/ns_$v.json 2> gpurun_out/ns_$v.err || exit 2
  python3 -c "import json;d=json.load(open('gpurun_out/ns_$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
done
