#!/bin/bash
# GPU test suite + Fitch/Sankoff bench lines (no CPU baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/gputests.log; exit 1; }
tail -1 gpurun_out/gputests.log
timeout -k 10 300 python bench.py --no-cpu --with none "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 2
timeout -k 10 300 python bench.py --no-cpu --with none --mode sankoff "$@" > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err || exit 3
python3 - <<'P'
import json
for f in ('gpurun_out/bench.json','gpurun_out/bench_s.json'):
    d=json.load(open(f)); r=d['roofline']
    print(f, 'ms', round(d['ms_per_step'],3), 'value %.3e'%d['value'], r['kernel'], 'launch_ms', r['avg_launch_ms'], 'kern_ms', r['kernel_ms_per_step'], r['other_kernels_ms_per_step'], 'score', r['score_kernel_ms_per_step'])
P
