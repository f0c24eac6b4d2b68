#!/bin/bash
# A round's evidence in up to three GPU calls (repo root on the box):
#   tools/round_evidence.sh profile TAG [PARTS]  -- the profile set (tools/profile_set.sh)
#   tools/round_evidence.sh merge TAG            -- (here) PMC traffic of every gpurun_out/prof_TAG*
#                                                   merged into profiles/traffic_fitch.json
#   tools/round_evidence.sh check TAG            -- every -m gpu test, the default bench line and
#                                                   the C3 / C4 (T2) lines against that traffic file
set -o pipefail
cd "$(dirname "$0")/.."
what=$1; tag=$2
case $what in
  profile) PARTS="${3:-}" bash tools/profile_set.sh $tag ;;
  merge) python3 tools/merge_traffic.py profiles/traffic_fitch.json $(ls -d gpurun_out/prof_${tag}*/traffic.json gpurun_out/prof_replay_${tag}/traffic.json 2>/dev/null) ;;
  check) bash tools/gpu_round_check.sh $tag ;;
esac
