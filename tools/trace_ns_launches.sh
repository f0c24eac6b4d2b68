#!/bin/bash
# Per-launch kernel trace of one N* Fitch step (GPU box): gpurun_out/ns_launches_TAG.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
tag=$1
out=gpurun_out/ns_trace_$tag
mkdir -p "$out"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$out" -o run -- python3 bench.py --no-cpu --with none --steps 3 --warmup 1 > "$out/bench.json" 2> "$out/bench.log" || exit 2
csv=$(find "$out" -name "*kernel_trace.csv" | head -1)
python3 tools/trace_launches.py "$csv" "k_" --step > gpurun_out/ns_launches_$tag.txt
echo "--- summary" >> gpurun_out/ns_launches_$tag.txt
python3 tools/trace_launches.py "$csv" "k_" --step --summary >> gpurun_out/ns_launches_$tag.txt
tail -12 gpurun_out/ns_launches_$tag.txt
