#!/bin/bash
# Round evidence, part B (GPU box): N* Sankoff profile, C3 / C3 Sankoff / C2 traces, replay PMC
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
bash tools/profile_fitch.sh ${tag}_sankoff --mode sankoff || exit 3
bash tools/trace_stats.sh ${tag}_c3 --tree sars-like --leaves 100000 --steps 5 --warmup 2 || exit 4
bash tools/trace_stats.sh ${tag}_c3_sankoff --tree sars-like --leaves 100000 --mode sankoff --steps 5 --warmup 2 || exit 5
bash tools/trace_stats.sh ${tag}_c2 --leaves 4096 --sites 15000 --steps 10 --warmup 3 || exit 6
bash tools/profile_replay.sh $tag || exit 7
