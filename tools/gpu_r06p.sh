#!/bin/bash
# N* Fitch profile set + C3 Fitch PMC (stats, FETCH, WRITE, SQ):  tools/gpu_r06p.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."
tag=$1
( while sleep 50; do echo "[hb] $(date +%T)"; done ) & hb=$!
trap "kill $hb" EXIT
bash tools/profile_fitch.sh $tag || exit 2
bash tools/profile_fitch.sh ${tag}_c3 --tree sars-like --leaves 100000 || exit 3
for d in $tag ${tag}_c3; do echo "== $d"; cat gpurun_out/prof_$d/traffic.txt; head -30 gpurun_out/prof_$d/sq.txt; done
