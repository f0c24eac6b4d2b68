#!/bin/bash
# r05i: N* Fitch per-launch trace (one step) + the replay bench lines with the new kernel names.
set -o pipefail
cd "$(dirname "$0")/.."
bash tools/trace_stats.sh r05i_ns --steps 2 --warmup 1 && \
python3 tools/trace_launches.py $(find gpurun_out/trace_r05i_ns -name "*kernel_trace.csv" | head -1) k_ --step > gpurun_out/trace_r05i_ns_launches.txt && \
timeout -k 10 300 python bench.py --mode replay --no-cpu --steps 10 --warmup 2 > gpurun_out/r05i_replay.json 2> gpurun_out/r05i_replay.err && \
python3 -c "import json;d=json.load(open('gpurun_out/r05i_replay.json'));print(d['ms_per_step'], json.dumps(d['roofline']))"
