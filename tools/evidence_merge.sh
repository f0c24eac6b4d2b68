#!/bin/bash
# Round evidence, local step between the GPU parts: the PMC traffic of parts A and B merged into
# profiles/traffic_fitch.json (what bench.py reports when the build id matches)
set -e
cd "$(dirname "$0")/.."
tag=$1
python3 tools/merge_traffic.py profiles/traffic_fitch.json gpurun_out/prof_$tag/traffic.json \
  gpurun_out/prof_${tag}_sankoff/traffic.json gpurun_out/prof_replay_$tag/traffic.json
