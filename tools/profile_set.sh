#!/bin/bash
# The round's profile set (GPU box, repo root): N* Fitch / Sankoff, C3 Fitch / Sankoff and
# (C4=1) the C4 rank share on the SARS-like tree -- rocprofv3 stats + FETCH / WRITE / SQ passes
# each, stamped with the build id -- the C2 kernel trace and the replay PMC.
#   tools/profile_set.sh TAG  ->  gpurun_out/{prof_TAG*, trace_TAG_c2, prof_replay_TAG}
#   PARTS="ns c3 c2 replay c4t2" picks a subset (default: all but c4t2)
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
mkdir -p gpurun_out
( while sleep 50; do echo "[hb] $(date +%T)"; done ) & hb=$!
trap "kill $hb" EXIT
parts=${PARTS:-ns c3 c2 replay}
for p in $parts; do
  case $p in
    ns) bash tools/profile_fitch.sh $tag && bash tools/profile_fitch.sh ${tag}_sankoff --mode sankoff || exit 2 ;;
    c3) bash tools/profile_fitch.sh ${tag}_c3 --tree sars-like --leaves 100000 &&
        bash tools/profile_fitch.sh ${tag}_c3_sankoff --tree sars-like --leaves 100000 --mode sankoff || exit 3 ;;
    c2) bash tools/trace_stats.sh ${tag}_c2 --leaves 4096 --sites 15000 --steps 10 --warmup 3 || exit 4 ;;
    replay) bash tools/profile_replay.sh $tag || exit 5 ;;
    c4t2) bash tools/profile_fitch.sh ${tag}_c4t2 --tree sars-like --leaves 8000000 --sites 3750 || exit 6 ;;
    c4) bash tools/trace_stats.sh ${tag}_c4 --leaves 8000000 --sites 3750 --steps 5 --warmup 2 || exit 7 ;;
  esac
  echo "profile part $p done"
done
echo "profile_set $tag done"
