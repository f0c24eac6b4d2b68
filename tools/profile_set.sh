#!/bin/bash
# The round's evidence set after a default bench (GPU box, repo root): N* Fitch / Sankoff
# rocprofv3 stats + PMC passes (stamped with the build id), C3 / C2 kernel traces, replay PMC.
#   tools/profile_set.sh TAG  ->  gpurun_out/{prof_TAG*, trace_TAG_*, prof_replay_TAG}
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
bash tools/profile_fitch.sh $tag || exit 2
bash tools/profile_fitch.sh ${tag}_sankoff --mode sankoff || exit 3
bash tools/trace_stats.sh ${tag}_c3 --tree sars-like --leaves 100000 --steps 5 --warmup 2 || exit 4
bash tools/trace_stats.sh ${tag}_c3_sankoff --tree sars-like --leaves 100000 --mode sankoff --steps 5 --warmup 2 || exit 5
bash tools/trace_stats.sh ${tag}_c2 --leaves 4096 --sites 15000 --steps 10 --warmup 3 || exit 6
bash tools/profile_replay.sh $tag || exit 7
echo "profile_set $tag done"
