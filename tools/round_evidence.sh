#!/bin/bash
# A round's evidence on one GPU box (repo root): the profile set, its PMC traffic merged into
# profiles/traffic_fitch.json (a copy lands in gpurun_out/), then every -m gpu test and the
# default bench line against that traffic file:
#   tools/round_evidence.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
bash tools/profile_set.sh $tag || exit 2
python3 tools/merge_traffic.py profiles/traffic_fitch.json gpurun_out/prof_$tag/traffic.json \
  gpurun_out/prof_${tag}_sankoff/traffic.json gpurun_out/prof_replay_$tag/traffic.json || exit 3
cp profiles/traffic_fitch.json gpurun_out/traffic_fitch_$tag.json
bash tools/gpu_round_check.sh $tag || exit 4
