#!/bin/bash
# N* Fitch kernel trace: every dispatch of the last step (post-order levels, pre-order, tail)
set -o pipefail
cd "$(dirname "$0")/.."
tag=${1:-r04b}
bash tools/trace_stats.sh ${tag}_ns --steps 2 --warmup 1 ${BENCH_ARGS:-} || exit 2
f=$(find gpurun_out/trace_${tag}_ns -name "*kernel_trace.csv" | head -1)
python3 tools/trace_launches.py "$f" k_fitch_up --last ${UP_LAUNCHES:-24} > gpurun_out/trace_${tag}_ns/up_launches.txt
python3 tools/trace_launches.py "$f" k_down --last ${DOWN_LAUNCHES:-40} > gpurun_out/trace_${tag}_ns/down_launches.txt
python3 tools/trace_launches.py "$f" k_tail --last 1 >> gpurun_out/trace_${tag}_ns/down_launches.txt
cat gpurun_out/trace_${tag}_ns/up_launches.txt
tail -3 gpurun_out/trace_${tag}_ns/down_launches.txt
